# Round-4 one-call GPU session: the -m gpu suite and the bench line (tools/gpu_r04.sh), the
# evidence (tools/gpu_evidence_r04.sh: PMC traffic + SQ counters + kernel stats), then the
# A/B of k_flow's per-wave small items (parity first) and of the inter-tile reference order.
# Each step time-limited; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
bash tools/gpu_r04.sh || exit $?
bash tools/gpu_evidence_r04.sh > gpurun_out/evidence.log 2>&1 || { tail -20 gpurun_out/evidence.log; exit 1; }
tail -25 gpurun_out/evidence.log
bash tools/gpu_r04_wave.sh || exit $?
bash tools/gpu_env_ab.sh AV1R_INTER_ORDER=1
