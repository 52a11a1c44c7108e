# Round 6 closing check at the tree's HEAD: the whole GPU suite, smoke(), then the default
# bench line (reading the committed PMC traffic, measured on identical kernels).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/final/pytest.log 2>&1 || { tail -40 gpurun_out/final/pytest.log; exit 1; }
tail -2 gpurun_out/final/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print(d['value'], d['device_only_fps'], d['recon_kernel_ms_per_frame'], d['key_frame_alone_ms']['recon'], d['config_4k']['value'] if 'config_4k' in d else '', d['ivf_end_to_end']['fps'], d['roofline']['frac'], d['cpu_baseline']['value'])"
