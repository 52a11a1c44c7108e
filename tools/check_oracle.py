import hashlib, sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from av1dec_amd import batchfile
import pyoracle, golden

names = sys.argv[1:] or golden.streams()
bm = golden.bits_md5()
bad = 0
for s in names:
    frames = batchfile.load(golden.batch_path(s))
    rows, outmd5 = golden.stage_hashes(s)
    o = pyoracle.Oracle()
    md = hashlib.md5()
    msg = ""
    t = time.time()
    for i, fr in enumerate(frames):
        o.decode_frame(fr)
        if not fr.show_existing:
            for st, name in enumerate(("recon", "lf", "cdef", "lr")):
                hsh = pyoracle.md5_planes(o.read_stage(st))
                if hsh != rows[i][3 + st] and not msg:
                    msg = f"frame {i} stage {name} mismatch"
        while o.output_pending():
            y, u, v = o.get_output()
            md.update(y.tobytes()); md.update(u.tobytes()); md.update(v.tobytes())
    ok = md.hexdigest() == outmd5 == bm.get(s)
    if not ok or msg:
        bad += 1
        print("FAIL", s, msg, md.hexdigest(), outmd5)
    else:
        print("ok  ", s, f"{time.time()-t:.2f}s")
print("bad", bad, "of", len(names))
