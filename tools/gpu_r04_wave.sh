# k_flow per-wave small items (AV1R_FLOW_WAVE=1): parity (the 172 conformance streams, stage by
# stage, and the headline pipeline), then the env A/B of bench.py against the default.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AV1R_FLOW_WAVE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_headline.py -m gpu -x -q \
    -k "matches_reference and not strip and not fused or headline_cycle" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/wavetest.log 2>&1 || { tail -30 gpurun_out/wavetest.log; exit 1; }
tail -2 gpurun_out/wavetest.log
bash tools/gpu_env_ab.sh AV1R_FLOW_WAVE=1
