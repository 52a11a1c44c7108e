"""Stress (GPU box): 8 decoders fed by 8 host threads (1080p synthetic streams), counting the
k_flow wait timeouts (concurrent threads and the flow chain).
usage: python3 tools/thr_stress.py [reps]   (PREWARM=1: one serial frame per context first)"""
import os, sys, threading, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools", "synth")]
import pysynth
from av1dec_amd import Decoder
S, N, REP = 8, 24, int(sys.argv[1]) if len(sys.argv) > 1 else 5
streams = [pysynth.stream(1920, 1080, N, 0x5EED1000 + i) for i in range(S)]
fails = 0
if os.environ.get("PREWARM"):  # (round 1 workaround probe; no longer needed)  # every context's buffers allocated before the threaded reps
    keep = [Decoder(0, keep_stages=False) for _ in range(S)]
    for d, fr in zip(keep, streams):
        d.decode_frame(fr[0]); d.synchronize()
    for d in keep: d.close()
for rep in range(REP):
    decs = [Decoder(0, keep_stages=False) for _ in range(S)]
    for d in decs:
        d.set_discard_output(True)
    errs = []
    def feed(d, fr):
        try:
            for f in fr:
                d.decode_frame(f)
            d.synchronize()
            d.decode_frame(fr[0]); d.synchronize()  # surfaces an error of the last launches
        except Exception as e:
            errs.append(str(e)[:120])
    th = [threading.Thread(target=feed, args=(d, fr)) for d, fr in zip(decs, streams)]
    t = time.perf_counter()
    for x in th: x.start()
    for x in th: x.join()
    dt = time.perf_counter() - t
    fails += bool(errs)
    import ctypes as C
    from av1dec_amd import native
    pairs, cross = (C.c_uint32 * 8)(), C.c_int()
    ov = native.lib().av1r_flow_debug(pairs, 8, 1, C.byref(cross))  # -1: not a -DAV1R_FLOW_DEBUG build
    print(f"gran={os.environ.get('AV1R_GRAN', '1')} rep {rep}: {dt:.2f} s, errors {len(errs)} {errs[:1]}; "
          f"k_flow overlapping entries {ov} (cross-stream pairs {cross.value}) {[hex(x) for x in pairs][:4]}", flush=True)
    for d in decs:
        try: d.close()
        except Exception as e: print("close:", e)
print("fails", fails)
