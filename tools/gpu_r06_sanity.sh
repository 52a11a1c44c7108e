cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s1
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s1/pytest.log 2>&1 || { tail -40 gpurun_out/s1/pytest.log; exit 1; }
tail -2 gpurun_out/s1/pytest.log
timeout -k 10 600 python3 bench.py --traffic profiles/traffic.json --traffic-4k profiles/traffic_4k.json > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/s1/bench.json')); print(d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['key_frame_alone_ms'], d['ivf_end_to_end']['fps'], d['ivf_end_to_end']['parse_ms_per_frame'])"
