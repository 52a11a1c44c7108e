# The bench's frame-delivery leg under delivery variants (one run each, no other legs):
# default, completion by the stream going idle (AV1R_OUT_SQ), each with the read-backs on
# a stream of their own (AV1R_OUT_ON_COPY=0).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/out2
for cfg in "X=0" "AV1R_OUT_SQ=1" "AV1R_OUT_SQ=1 AV1R_OUT_ON_COPY=0" "AV1R_OUT_ON_COPY=0" "X=0" "AV1R_OUT_SQ=1"; do
    env $cfg timeout -k 10 300 python3 bench.py --no-cpu --ivf-frames 0 --no-4k > gpurun_out/out2/b.json 2> gpurun_out/out2/b.err || { tail -5 gpurun_out/out2/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/out2/b.json')); o=d['output_inclusive']; print('$cfg', d['value'], o['fps'], o['vs_headline'], o['launcher_output_ms_per_step'])"
done
