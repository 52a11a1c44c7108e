#!/usr/bin/env python3
"""Frame-delivery probe (A/B aid): 8 synthetic 1080p streams (GOP phases staggered as in
bench.py) through one native pipeline, with or without the pinned ring sink
(av1r_pipeline_set_output); prints the rate, the launcher's split and the monotonic-clock
window of the timed step (to cut a rocprofv3 trace to it).
usage: python3 tools/out_probe.py [frames] [steps] [out|none]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def main():
    import bench
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import NativePipeline, RingSink
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 120
    out = (sys.argv[3] if len(sys.argv) > 3 else "out") == "out"
    S = 8
    streams = bench.rank_streams("1080p", 0, S, F)
    decs = [Decoder(0, keep_stages=False) for _ in streams]
    for d in decs:
        d.set_discard_output(not out)
    pp = bench.StreamScheduler(decs, F, streams=streams, workers=1)
    pp.stagger()  # stream j decoded alone up to frame j*F/S
    pp.close()
    for d in decs:
        d.synchronize()
    sink = RingSink(S, 1920, 1080) if out else None
    pl = NativePipeline(decs, streams, list(pp.pos), depth=0, workers=bench.host_workers())
    try:
        if sink:
            pl.set_output(sink)
        pl.step(F)
        n0 = sink.delivered() if sink else 0
        t0 = time.perf_counter()
        m0 = time.monotonic_ns()
        st = pl.step(steps)
        dt = time.perf_counter() - t0
        print("window_ns", m0, time.monotonic_ns())
        print({"fps": round(S * steps / dt, 1), "output_ms_per_step": round(1e3 * st["output_s"] / steps, 3),
               "launch_ms_per_step": round(1e3 * st["launch_s"] / steps, 3),
               "idle_ms_per_step": round(1e3 * st["wait_s"] / steps, 3), "batches": int(st["batches"]),
               "delivered": (sink.delivered() - n0) if sink else 0})
        if sink:
            pl.set_output(None)
    finally:
        pl.close()
        if sink:
            sink.close()
        for d in decs:
            d.close()


if __name__ == "__main__":
    main()
