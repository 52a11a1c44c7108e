# Round-4 check at the current tree in one call: the -m gpu suite, then the bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
timeout -k 10 500 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { tail -30 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json
b = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
print("value", b["value"], "device_only", b["device_only_fps"], "out", (b.get("output_inclusive") or {}).get("fps"),
      "stage", b["stage_ms_per_frame"], "kern", b["recon_kernel_ms_per_frame"], "4k", (b.get("config_4k") or {}).get("fps"),
      "ivf", (b.get("ivf_end_to_end") or {}).get("fps"), "kf", b["key_frame_alone_ms"])
PY
