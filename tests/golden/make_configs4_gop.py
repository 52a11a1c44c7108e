#!/usr/bin/env python3
"""Golden output hashes of BASELINE configs[4]'s 64 synthetic 1080p streams over a whole GOP
(60 frames each: 1 key + 59 inter), from the CPU oracle (oracle/pyoracle, the restatement
pinned against the reference decoder) on the same batches bench.rank_streams builds.
One line per stream id: 60 hex digests, each md5 over the concatenated md5 digests of the
frame's Y, U and V planes (tests/test_multi.py's md5s).  Test infrastructure: the GPU test
test_gpu_configs4_whole_gop_matches_golden decodes the same streams and compares.

usage: python tests/golden/make_configs4_gop.py   (CPU only; ~8 processes, several minutes)"""
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "tests", "golden", "configs4_gop_md5.json")
S, F, WORLD = 8, 60, 8


def one_rank(rank):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bench
    import pyoracle
    ids = bench.rank_stream_ids(rank, S)
    streams = bench.rank_streams("1080p", rank, S, F)
    res = {}
    for sid, frames in zip(ids, streams):
        o = pyoracle.Oracle(keep_stages=False)
        out = []
        try:
            for f in frames:
                o.decode_frame(f)
                while o.output_pending():
                    planes = o.get_output()
                    out.append(hashlib.md5(b"".join(hashlib.md5(p.tobytes()).digest() for p in planes)).hexdigest())
        finally:
            o.close()
        res[str(sid)] = out
    return res


def main():
    allr = {}
    with ProcessPoolExecutor(int(os.environ.get("JOBS", "8"))) as ex:
        for r in ex.map(one_rank, range(WORLD)):
            allr.update(r)
    assert sorted(int(k) for k in allr) == list(range(S * WORLD))
    json.dump({"streams": S * WORLD, "frames": F, "config": "1080p", "hash": "md5(md5(Y) | md5(U) | md5(V))",
               "md5": allr}, open(OUT, "w"), indent=0, sort_keys=True)
    print(OUT, sum(len(v) for v in allr.values()), "frames")


if __name__ == "__main__":
    main()
