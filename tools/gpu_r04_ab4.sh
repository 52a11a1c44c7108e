# Frame-delivery breakdown: the probe's launcher split (AV1R_PIPE_PROF) and its HIP API trace
# over the timed window, then the bench's output leg.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
AV1R_PIPE_PROF=1 timeout -k 10 200 python3 tools/out_probe.py 12 400 > gpurun_out/ab4/probe.log 2>&1 || { tail -5 gpurun_out/ab4/probe.log; exit 1; }
grep -E "fps|outputs|window" gpurun_out/ab4/probe.log
timeout -k 10 200 rocprofv3 --hip-trace --output-format csv -d gpurun_out/ab4/ht -o run -- python3 tools/out_probe.py 12 400 > gpurun_out/ab4/ht.log 2>&1 || { tail -5 gpurun_out/ab4/ht.log; exit 1; }
grep -E "fps|window" gpurun_out/ab4/ht.log
timeout -k 10 300 python3 bench.py --steps 60 --warmup 5 --no-cpu --ivf-frames 0 --no-4k --output-steps 120 > gpurun_out/ab4/run.json 2> gpurun_out/ab4/run.err || { tail -5 gpurun_out/ab4/run.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab4/run.json')); o=d['output_inclusive']; print(d['value'], d['host_profile']); print('  out', {k: v for k, v in o.items() if k != 'method'})"
