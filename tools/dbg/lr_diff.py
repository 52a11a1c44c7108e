"""Debug aid: where the GPU's loop-restoration stage differs from the oracle's on frame 0."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import golden, pyoracle
from av1dec_amd import Decoder, batchfile, abi
for s in sys.argv[1:]:
    fr = batchfile.load(golden.batch_path(s))[0]
    h = fr.hdr
    d = Decoder(0, keep_stages=True)
    d.decode_frame(fr)
    g = d.read_stage(3)
    o = pyoracle.Oracle(keep_stages=True)
    o.decode_frame(fr)
    ref = o.read_stage(3) if hasattr(o, "read_stage") else None
    print(s, "lr types", list(h.lr_type), "unit sizes", list(h.lr_unit_size), "size", h.frame_width, h.frame_height)
    lr = np.frombuffer(fr.sec["lr"].tobytes(), abi.LR_DTYPE) if hasattr(abi, "LR_DTYPE") else None
    if lr is not None:
        print(" unit types", np.bincount(lr["type"], minlength=3))
    for p in range(3):
        a, b = g[p], ref[p]
        dd = np.argwhere(a != b)
        print(" plane", p, "diffs", len(dd), "of", a.size)
        if len(dd):
            ys, xs = dd[:, 0], dd[:, 1]
            print("  x%64 hist", np.bincount(xs % 64, minlength=64).tolist())
            print("  y range", ys.min(), ys.max(), "x range", xs.min(), xs.max(), "first", dd[:5].tolist(), a[tuple(dd[0])], b[tuple(dd[0])])
    d.close(); o.close()
