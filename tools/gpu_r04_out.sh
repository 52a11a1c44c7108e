# The bench's frame-delivery leg at its default length, three times (spread), no other legs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/out
OUT_ENV=${OUT_ENV:-X=0}
for i in 1 2 3; do
    env $OUT_ENV timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k > gpurun_out/out/b$i.json 2> gpurun_out/out/b$i.err || { tail -5 gpurun_out/out/b$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/out/b$i.json')); o=d['output_inclusive']; print(d['value'], o['fps'], o['vs_headline'], o['elapsed_s'], o['launcher_output_ms_per_step'])"
done
