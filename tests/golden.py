"""Access to the committed golden fixtures (tests/golden/), produced from the reference
decoder by tools/make_golden.py: frame batches, per-stage MD5s and bits.md5."""
import os

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def streams():
    d = os.path.join(GOLD, "batches")
    return sorted(f[:-len(".av1b.gz")] for f in os.listdir(d) if f.endswith(".av1b.gz"))


def batch_path(stream):
    return os.path.join(GOLD, "batches", stream + ".av1b.gz")


def stage_hashes(stream):
    """[(frame_type, show_frame, show_existing, recon, lf, cdef, lr)], output_md5"""
    rows, out = [], None
    with open(os.path.join(GOLD, "hashes", stream + ".txt")) as f:
        for line in f:
            p = line.split()
            if p[0] == "md5":
                out = p[1]
            else:
                rows.append((int(p[1]), int(p[2]), int(p[3]), p[4], p[5], p[6], p[7]))
    return rows, out


def bits_md5():
    m = {}
    with open(os.path.join(GOLD, "bits.md5")) as f:
        for line in f:
            p = line.split()
            if len(p) == 2:
                m[p[1].replace(".ivf", "").replace(".mkv", "")] = p[0]
    return m


REF_BITS = os.path.join(os.environ.get("AV1DEC_REF", "/root/reference"), "bits")


def ivf_path(stream):
    """The conformance bitstream itself: the reference checkout's bits/<stream>.ivf.  Only in
    the build container -- the bitstreams are not part of this repository, so tests that
    parse them are CPU tests that skip where the checkout is absent."""
    return os.path.join(REF_BITS, stream + ".ivf")


def have_ivf():
    return os.path.isdir(REF_BITS)
