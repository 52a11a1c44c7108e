# A/B of the native launcher's stream groups (AV1R_PIPE_GROUPS) after a parity check of the
# k_mi change (stage-exact on the conformance streams + the native pipeline tests).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "test_gpu_matches_reference or native or packed" > gpurun_out/ab/parity.log 2>&1 || { tail -30 gpurun_out/ab/parity.log; exit 1; }
tail -1 gpurun_out/ab/parity.log
for g in 1 2 4 1 2; do
    AV1R_PIPE_GROUPS=$g timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --steps 60 > gpurun_out/ab/g$g.json 2> gpurun_out/ab/g$g.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/g$g.json')); print('groups $g', d['value'], d['device_only_fps'], d['host_profile'])"
done
