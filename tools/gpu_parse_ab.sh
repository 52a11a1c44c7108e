# Host parser A/B on the GPU box's CPU (steadier than the build container): parse_bench
# binaries built here (tools/_build/parse_ab/pb_*: tools/parse_bench.cpp against different
# trees or flags) on the same 1080p_s1 IVF, alternately, single-threaded, CPU time, best of 10.
cd $GRAFT_REPO_ROOT
d=tools/_build/parse_ab
for r in 1 2 3; do
    for b in $d/pb_*; do
        echo -n "$(basename $b): "; AV1P_CPU_TIME=1 AV1P_NO_MI=1 AV1P_TILE_THREADS=1 timeout -k 5 120 $b $d/s1.ivf 10 || exit 1
    done
done
