# k_flow per-wave small items (av1r_set_flow_wave / AV1R_FLOW_WAVE=1): its parity tests (the
# A/B subset of the conformance streams stage by stage, synthetic 1080p and 4K), the headline
# pipeline with it, then the env A/B of bench.py against the default.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_synth.py -m gpu -x -q -k "flow_wave" \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/wavetest.log 2>&1 || { tail -30 gpurun_out/wavetest.log; exit 1; }
AV1R_FLOW_WAVE=1 timeout -k 10 400 python -u -m pytest tests/test_headline.py -m gpu -x -q -k "headline_cycle" \
    --timeout 300 --timeout-method thread -p no:cacheprovider >> gpurun_out/wavetest.log 2>&1 || { tail -30 gpurun_out/wavetest.log; exit 1; }
tail -2 gpurun_out/wavetest.log
bash tools/gpu_env_ab.sh AV1R_FLOW_WAVE=1
