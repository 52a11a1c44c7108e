# GPU parity of the current build, then the 1080p + 4K bench in rotation (twice) over the
# current build and alternatives: each argument is either a .so path (AV1R_LIB) or an
# environment setting VAR=value.  usage: bash tools/gpu_ab3.sh alt.so "AV1R_X=1" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in "" "$@"; do
    case "$v" in *.so) e="AV1R_LIB=$v";; *) e="$v";; esac
    env $e timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --ivf-frames 0 --output-steps 0 \
        > gpurun_out/ab3/run.json 2> gpurun_out/ab3/run.err || { tail -5 gpurun_out/ab3/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab3/run.json')); k=d['config_4k']; print('${v:-current}', d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['stage_ms_per_frame'], d['key_frame_alone_ms']['recon'], '4k', k['fps'], k['device_only_fps'], k['recon_kernel_ms_per_frame'])"
  done
done
