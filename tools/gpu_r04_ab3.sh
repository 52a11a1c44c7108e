# Frame-delivery A/B: the output leg's launcher profile next to the headline's.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3
for cfg in "" "AV1R_OUT_NOCOPY=1 AV1R_OUT_NOREADY=1"; do
    env $cfg timeout -k 10 300 python3 bench.py --steps 60 --warmup 5 --no-cpu --ivf-frames 0 --no-4k --output-steps 120 > gpurun_out/ab3/run.json 2> gpurun_out/ab3/run.err || { tail -5 gpurun_out/ab3/run.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab3/run.json')); o=d['output_inclusive']; print('${cfg:-default}', d['value'], d['host_profile']); print('  out', {k: v for k, v in o.items() if k != 'method'})"
done
