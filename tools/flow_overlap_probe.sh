# Known-issue probe: the threaded stress on the -DAV1R_FLOW_DEBUG build, which
# counts k_flow workgroup entries that find another launch's workgroups still running
cd $GRAFT_REPO_ROOT
for r in 1 2 3 4 5; do
  AV1R_LIB=av1dec_amd/_build/libflowdbg.so timeout -k 10 200 python tools/thr_stress.py 2 > gpurun_out/ov_$r.txt 2>&1 || exit $?
  echo "run $r: $(grep -h "errors [1-9]" gpurun_out/ov_$r.txt | cut -c1-60 | tr '\n' ' ') $(grep -h "co-resident" gpurun_out/ov_$r.txt | tail -1)"
done
