# Round 6: LF unit compaction (AV1R_LF_COMPACT=1, the filtering units packed to a workgroup's
# first lanes): the whole GPU suite with it, then the headline A/B against the uncompacted build.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lfc
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/lfc/pytest.log 2>&1 || { tail -40 gpurun_out/lfc/pytest.log; exit 1; }
tail -1 gpurun_out/lfc/pytest.log
R=3 bash tools/gpu_r06_libab.sh av1dec_amd/_build/libav1r_lfc0.so
