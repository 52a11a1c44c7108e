import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tools", "synth"))
import pysynth
from av1dec_amd import Decoder
S, F = 8, 60
streams = [pysynth.stream(1920, 1080, F, 0x5EED1000 + j) for j in range(S)]
decs = [Decoder(0, keep_stages=False, timing=False) for _ in range(S)]
for d in decs: d.set_discard_output(True)
hs = [[d.prepare(f) for f in fr] for d, fr in zip(decs, streams)]
def step(t): Decoder.decode_prepared_batch(decs, [h[t % F] for h in hs])
for t in range(2 * F): step(t)
for d in decs: d.synchronize()
for rep in range(3):
    t0 = time.perf_counter(); per = []
    for t in range(F):
        a = time.perf_counter(); step(t); per.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    for d in decs: d.synchronize()
    t2 = time.perf_counter()
    per.sort()
    print(f"issue {1e3*(t1-t0):.1f} ms, total {1e3*(t2-t0):.1f} ms, per-step call p50 {1e6*per[len(per)//2]:.0f} us p90 {1e6*per[int(len(per)*0.9)]:.0f} us max {1e6*per[-1]:.0f}")
for d in decs: d.close()
