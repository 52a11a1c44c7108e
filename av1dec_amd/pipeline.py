"""Many independent AV1 streams decoded end to end on one GPU.

Each stream gets a host thread that parses its temporal units in order (av1p_decode_tu, the
host parser linked into libav1r.so) and packs every completed frame (av1r_pack: validation,
dependency schedule, pinned copy) into that stream's queue, a few frames ahead.  One launching
thread takes the next packed frame of every stream that has one and is not running a key frame
alone (av1r_busy), and decodes them in shared launches (av1r_decode_packed_batch).  Parse of
frame N+1 therefore overlaps the GPU work of frame N (legal: parsing needs only the previous
frames' parse state, never their pixels -- SURVEY K4), and the streams' parses run in parallel.

This is the reference's Decoder::decode loop (decoder/Av1Decoder.cpp:49-109) per stream, with
the per-frame reconstruction (Av1Decoder.cpp:128-192) batched across streams."""
import ctypes as C
import queue
import threading
import time

from . import native
from .decoder import BackendError, Decoder
from .parser import ivf_frames


def _plib():
    l = native.lib()  # libav1r.so carries the parser too (include/av1p.h)
    vp = C.c_void_p
    l.av1p_create.argtypes = [C.POINTER(vp)]
    l.av1p_destroy.argtypes = [vp]
    l.av1p_destroy.restype = None
    l.av1p_decode_tu.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
    l.av1p_frame.argtypes = [vp, C.c_int]
    l.av1p_frame.restype = vp
    l.av1p_last_error.argtypes = [vp]
    l.av1p_last_error.restype = C.c_char_p
    l.av1p_set_mode_info.argtypes = [vp, C.c_int]
    return l


class IvfPipeline:
    """streams: IVF file contents (bytes), one per stream; decoders: one Decoder each (same
    device).  run() decodes every frame of every stream once and returns the elapsed seconds."""

    def __init__(self, decoders, streams, depth=3):
        if len(decoders) != len(streams):
            raise ValueError("one decoder per stream")
        self.decs, self.depth = decoders, depth
        self.tus = [list(ivf_frames(s)) for s in streams]
        self.l = _plib()
        self.parse_s = [0.0] * len(streams)
        self.pack_s = [0.0] * len(streams)
        self.frames = [0] * len(streams)
        self.batches = 0

    def _producer(self, j, q, err):
        l = self.l
        p = C.c_void_p()
        if l.av1p_create(C.byref(p)):
            err.append("av1p_create failed")
            q.put(None)
            return
        l.av1p_set_mode_info(p, 0)  # the mode-info grid is rebuilt on the device (k_mi)
        n = C.c_int()
        try:
            for tu in self.tus[j]:
                t0 = time.perf_counter()
                rc = l.av1p_decode_tu(p, tu, len(tu), C.byref(n))
                t1 = time.perf_counter()
                self.parse_s[j] += t1 - t0
                if rc:
                    err.append(f"stream {j}: parse failed ({rc}): {l.av1p_last_error(p).decode()}")
                    return
                for i in range(n.value):
                    ptr = l.av1p_frame(p, i)
                    pk = C.c_void_p()
                    t2 = time.perf_counter()
                    rc = l.av1r_pack(ptr, C.byref(pk))
                    self.pack_s[j] += time.perf_counter() - t2
                    if rc:
                        err.append(f"stream {j}: av1r_pack failed ({rc}): {l.av1r_pack_last_error().decode()}")
                        return
                    q.put(pk)
                    self.frames[j] += 1
        finally:
            l.av1p_destroy(p)
            q.put(None)  # end of stream

    def run(self):
        S = len(self.decs)
        qs = [queue.Queue(maxsize=self.depth) for _ in range(S)]
        err = []
        th = [threading.Thread(target=self._producer, args=(j, qs[j], err), daemon=True) for j in range(S)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        live = set(range(S))
        head = [None] * S  # a packed frame taken from the queue, not yet launched
        try:
            while live and not err:
                for j in list(live):
                    if head[j] is None:
                        try:
                            head[j] = qs[j].get_nowait()
                        except queue.Empty:
                            continue
                        if head[j] is None:  # end of stream
                            live.discard(j)
                ready = [j for j in live if head[j] is not None and not self.decs[j].busy()]
                if not ready:
                    time.sleep(50e-6)
                    continue
                Decoder.decode_packed_batch([self.decs[j] for j in ready], [head[j] for j in ready])
                self.batches += 1
                for j in ready:
                    Decoder.free_packed(head[j])
                    head[j] = None
            for d in self.decs:
                d.synchronize()
        finally:
            for j in range(S):  # drain the producers (an error ends the run early)
                if head[j] is not None:
                    Decoder.free_packed(head[j])
                while th[j].is_alive() or not qs[j].empty():
                    try:
                        pk = qs[j].get(timeout=0.05)
                    except queue.Empty:
                        continue
                    if pk is not None:
                        Decoder.free_packed(pk)
            for t in th:
                t.join()
        if err:
            raise BackendError(err[0])
        return time.perf_counter() - t0


def _cycle_source(l, streams, positions, keep):
    n = len(streams)
    rows = []
    for fr in streams:
        arr = (C.c_void_p * len(fr))(*[C.cast(f.byref(), C.c_void_p).value for f in fr])
        rows.append(arr)
    table = (C.c_void_p * n)(*[C.cast(r, C.c_void_p).value for r in rows])
    count = (C.c_int * n)(*[len(fr) for fr in streams])
    pos = (C.c_int64 * n)(*(positions or [0] * n))
    cyc = native.Cycle(C.cast(table, C.c_void_p).value, count, pos, n)
    keep += [rows, table, count, pos, cyc, streams]
    src = native.StreamSource()
    src.next = C.cast(l.av1r_cycle_next, C.c_void_p).value
    src.user = C.cast(C.pointer(cyc), C.c_void_p).value
    src.stable = 1
    return src


class NativePipeline:
    """av1r_pipeline_open / _step / _close over a cycling source: the packing workers stay
    up between steps, `depth` frames ahead of every stream, so each step after the first
    runs in steady state (bench.py's headline).  positions: each stream's starting frame;
    positions() reports where every stream's launches have reached."""

    def __init__(self, decoders, streams, positions=None, depth=0, workers=0):
        self.l = l = native.lib()
        self.decs = decoders
        n = len(decoders)
        self.n = n
        self.pos0 = list(positions or [0] * n)
        self.keep = []
        self.src = _cycle_source(l, streams, self.pos0, self.keep)
        ctxs = (C.c_void_p * n)(*[d.c.value for d in decoders])
        self.keep.append(ctxs)
        self.p = C.c_void_p()
        rc = l.av1r_pipeline_open(ctxs, n, C.byref(self.src), int(depth), int(workers), C.byref(self.p))
        if rc:
            raise BackendError(f"av1r_pipeline_open failed ({rc})")

    def step(self, frames):
        """Launch `frames` more frames of every stream and synchronize; the step's stats."""
        st = native.PipelineStats()
        rc = self.l.av1r_pipeline_step(self.p, int(frames), C.byref(st))
        if rc:
            raise BackendError(f"av1r_pipeline_step failed ({rc}): {self.decs[0].l.av1r_last_error(self.decs[0].c).decode()}")
        return {k: getattr(st, k) for k, _ in native.PipelineStats._fields_}

    def set_output(self, sink):
        """Frame delivery (av1r_pipeline_set_output): a RingSink / ArraySink, or None."""
        self.sink = sink
        rc = self.l.av1r_pipeline_set_output(self.p, C.byref(sink.s) if sink is not None else None)
        if rc:
            raise BackendError(f"av1r_pipeline_set_output failed ({rc})")

    def positions(self):
        c = (C.c_int64 * self.n)()
        if self.l.av1r_pipeline_launched(self.p, c, self.n):
            raise BackendError("av1r_pipeline_launched failed")
        return [p0 + int(v) for p0, v in zip(self.pos0, c)]

    def close(self):
        if self.p:
            self.l.av1r_pipeline_close(self.p)
            self.p = C.c_void_p()


def run_native(decoders, source="cycle", streams=None, positions=None, max_frames=0, depth=0, workers=0):
    """The same pipeline in native threads (av1r_pipeline_run, include/av1r.h): no
    interpreter on the path (`workers` packing threads, 0: one per stream).  source "cycle": streams = per-stream lists of batchfile.Frame;
    stream j continues at frame positions[j] (mod its length), and positions is advanced in
    place by the frames decoded (it never ends: max_frames > 0 is required); "ivf": streams =
    IVF file contents.  Returns the
    av1r_pipeline_stats as a dict."""
    l = native.lib()
    n = len(decoders)
    ctxs = (C.c_void_p * n)(*[d.c.value for d in decoders])
    src = native.StreamSource()
    keep = []  # buffers the native side points into, alive for the call
    if source == "cycle":
        rows = []
        for fr in streams:
            arr = (C.c_void_p * len(fr))(*[C.cast(f.byref(), C.c_void_p).value for f in fr])
            rows.append(arr)
        table = (C.c_void_p * n)(*[C.cast(r, C.c_void_p).value for r in rows])
        count = (C.c_int * n)(*[len(fr) for fr in streams])
        pos = (C.c_int64 * n)(*(positions or [0] * n))
        if max_frames <= 0:
            raise ValueError("the cycle source never ends: max_frames must be > 0")
        cyc = native.Cycle(C.cast(table, C.c_void_p).value, count, pos, n)
        keep += [rows, table, count, pos, cyc, streams]
        src.next = C.cast(l.av1r_cycle_next, C.c_void_p).value
        src.user = C.cast(C.pointer(cyc), C.c_void_p).value
        src.stable = 1
    elif source == "ivf":
        bufs = [C.create_string_buffer(bytes(s), len(s)) for s in streams]
        files = (C.c_void_p * n)(*[C.cast(b, C.c_void_p).value for b in bufs])
        sizes = (C.c_size_t * n)(*[len(s) for s in streams])
        keep += [bufs, files, sizes]
        rc = l.av1r_ivf_source_create(files, sizes, n, C.byref(src))
        if rc:
            raise BackendError(f"av1r_ivf_source_create failed ({rc})")
    else:
        raise ValueError(source)
    st = native.PipelineStats()
    try:
        rc = l.av1r_pipeline_run(ctxs, n, C.byref(src), int(max_frames), int(depth), int(workers), C.byref(st))
    finally:
        if source == "ivf":
            l.av1r_ivf_source_destroy(C.byref(src))
    if rc:
        raise BackendError(f"av1r_pipeline_run failed ({rc}): {decoders[0].l.av1r_last_error(decoders[0].c).decode()}")
    if source == "cycle" and positions is not None:
        # every producer fetched exactly the frames that were decoded (max_frames each)
        positions[:] = list(pos)
    return {k: getattr(st, k) for k, _ in native.PipelineStats._fields_}


class RingSink:
    """The library's pinned-buffer output sink (av1r_ring_sink_create): `slots` frames of at
    most width x height per stream, reused in rotation; counts the frames delivered."""

    def __init__(self, n_streams, width, height, slots=native.SINK_INFLIGHT * 2):
        self.l = native.lib()
        self.s = native.OutputSink()
        rc = self.l.av1r_ring_sink_create(n_streams, width, height, slots, C.byref(self.s))
        if rc:
            raise BackendError(f"av1r_ring_sink_create failed ({rc})")
        self.n = n_streams

    def delivered(self, stream=None):
        if stream is None:
            return sum(self.delivered(j) for j in range(self.n))
        return int(self.l.av1r_ring_sink_delivered(C.byref(self.s), stream))

    def frame(self, stream, k):
        """Copies of the I420 planes of delivered frame k of `stream` (None once its slot has
        been reused; av1r_ring_sink_frame)."""
        import numpy as np
        w, h = C.c_int(), C.c_int()
        p = self.l.av1r_ring_sink_frame(C.byref(self.s), stream, k, C.byref(w), C.byref(h))
        if not p:
            return None
        W, H = w.value, h.value
        st, off, span = (C.c_int * 3)(), (C.c_size_t * 3)(), C.c_size_t()
        self.l.av1r_frame_layout(W, H, st, off, C.byref(span))  # the slot's layout
        a = np.ctypeslib.as_array((C.c_uint8 * span.value).from_address(p))
        out = []
        for q, (pw, ph) in enumerate(((W, H), (W >> 1, H >> 1), (W >> 1, H >> 1))):
            rows = np.lib.stride_tricks.as_strided(a[off[q]:], (ph, pw), (st[q], 1))
            out.append(rows.copy())
        return tuple(out)

    def close(self):
        if self.s.user:
            self.l.av1r_ring_sink_destroy(C.byref(self.s))


class ArraySink:
    """An output sink in Python (tests): every delivered frame kept as numpy I420 planes, per
    stream in delivery order, with its status."""

    def __init__(self, n_streams):
        import numpy as np
        self.np = np
        self.frames = [[] for _ in range(n_streams)]
        self.status = [[] for _ in range(n_streams)]
        self.inflight = [[] for _ in range(n_streams)]
        self._acq = native.SINK_ACQUIRE(self._acquire)
        self._del = native.SINK_DELIVER(self._deliver)
        self.s = native.OutputSink(C.cast(self._acq, C.c_void_p).value, C.cast(self._del, C.c_void_p).value, None)

    def _acquire(self, user, stream, w, h, planes, strides):
        np = self.np
        y = np.empty((h, w), np.uint8)
        u = np.empty(((h + 1) >> 1, (w + 1) >> 1), np.uint8)
        v = np.empty(((h + 1) >> 1, (w + 1) >> 1), np.uint8)
        self.inflight[stream].append((y, u, v))
        for k, a in enumerate((y, u, v)):
            planes[k] = a.ctypes.data
            strides[k] = a.strides[0]
        return 0

    def _deliver(self, user, stream, status):
        self.frames[stream].append(self.inflight[stream].pop(0))
        self.status[stream].append(status)
