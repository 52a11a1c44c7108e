"""Host-side mirror of the reference decoder API on top of the HIP backend.

`Decoder` follows YamiAv1::Decoder (decoder/Av1Decoder.h:47-66): frames go in,
`get_output()` pops shown frames in order or returns None (Av1Decoder.cpp:203-211).
What goes in is the frame batch the host parser produces for each decoded frame (the
reference's parsed Tile trees, see include/av1r.h), not OBU bytes."""
import ctypes as C

import numpy as np

from . import abi, native


class BackendError(RuntimeError):
    pass


class Decoder:
    def __init__(self, device=0, keep_stages=False, timing=False):
        self.l = native.lib()
        self.c = C.c_void_p()
        rc = self.l.av1r_create(device, C.byref(self.c))
        if rc != 0:
            raise BackendError(f"av1r_create({device}) failed: {rc}")
        self.l.av1r_set_keep_stages(self.c, int(keep_stages))
        self.l.av1r_set_timing(self.c, int(timing))
        self.last = None

    def close(self):
        if self.c:
            self.l.av1r_destroy(self.c)
            self.c = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            msg = self.l.av1r_last_error(self.c).decode()
            raise BackendError(f"{what} failed ({rc}): {msg}")

    def decode_frame(self, frame):
        """frame: batchfile.Frame (keeps its buffers alive)."""
        self.last = frame.hdr
        self._check(self.l.av1r_decode_frame(self.c, C.cast(frame.byref(), C.c_void_p)), "av1r_decode_frame")

    def decode_tiles(self, frame_level, tiles):
        self._check(self.l.av1r_frame_begin(self.c, C.cast(frame_level.byref(), C.c_void_p)), "av1r_frame_begin")
        for t in tiles:
            self._check(self.l.av1r_submit_tile(self.c, C.cast(t.byref(), C.c_void_p)), "av1r_submit_tile")
        self._check(self.l.av1r_frame_end(self.c), "av1r_frame_end")

    def prepare(self, frame):
        """Validate, schedule and upload a frame batch to HBM; returns a handle."""
        h = C.c_int()
        self._check(self.l.av1r_prepare(self.c, C.cast(frame.byref(), C.c_void_p), C.byref(h)), "av1r_prepare")
        return h.value

    def decode_prepared(self, handle):
        self._check(self.l.av1r_decode_prepared(self.c, handle), "av1r_decode_prepared")

    @staticmethod
    def decode_prepared_batch(decoders, handles):
        """One frame per decoder (independent streams, one device) in shared launches
        (av1r_decode_prepared_batch); launched on decoders[0]'s stream."""
        n = len(decoders)
        if n == 0 or n != len(handles):
            raise ValueError("need one handle per decoder")
        ctxs = (C.c_void_p * n)(*[d.c.value for d in decoders])
        hs = (C.c_int * n)(*handles)
        decoders[0]._check(decoders[0].l.av1r_decode_prepared_batch(ctxs, hs, n), "av1r_decode_prepared_batch")

    @staticmethod
    def pack(frame):
        """Validate, schedule and pack a frame batch into pinned host memory (av1r_pack:
        no context needed, safe from any thread).  Returns a handle for
        decode_packed_batch; free it with free_packed once that call has returned."""
        l = native.lib()
        p = C.c_void_p()
        rc = l.av1r_pack(C.cast(frame.byref(), C.c_void_p), C.byref(p))
        if rc != 0:
            raise BackendError(f"av1r_pack failed ({rc}): {l.av1r_pack_last_error().decode()}")
        return p

    @staticmethod
    def free_packed(p):
        native.lib().av1r_packed_free(p)

    @staticmethod
    def decode_packed_batch(decoders, packed):
        """Frame packed[i] of decoders[i] (independent streams, one device): uploaded from
        pinned memory and decoded in shared launches on decoders[0]'s stream."""
        n = len(decoders)
        if n == 0 or n != len(packed):
            raise ValueError("need one packed frame per decoder")
        ctxs = (C.c_void_p * n)(*[d.c.value for d in decoders])
        ps = (C.c_void_p * n)(*[p.value for p in packed])
        decoders[0]._check(decoders[0].l.av1r_decode_packed_batch(ctxs, ps, n), "av1r_decode_packed_batch")

    def busy(self):
        """True while a deep frame (key frame) of this decoder launched alone is running."""
        return self.l.av1r_busy(self.c) == 1

    def release_prepared(self, handle):
        self._check(self.l.av1r_release_prepared(self.c, handle), "av1r_release_prepared")

    def set_discard_output(self, discard):
        self._check(self.l.av1r_set_discard_output(self.c, int(discard)), "av1r_set_discard_output")

    def synchronize(self):
        self._check(self.l.av1r_synchronize(self.c), "av1r_synchronize")

    def output_pending(self):
        return self.l.av1r_output_pending(self.c)

    def get_output(self):
        w, h = C.c_int(), C.c_int()
        if self.l.av1r_get_output(self.c, None, 0, None, 0, None, 0, C.byref(w), C.byref(h)) != 0:
            return None
        W, H = w.value, h.value
        y = np.empty((H, W), np.uint8)
        u = np.empty((H >> 1, W >> 1), np.uint8)
        v = np.empty((H >> 1, W >> 1), np.uint8)
        self._check(self.l.av1r_get_output(self.c, y.ctypes.data, W, u.ctypes.data, W >> 1, v.ctypes.data,
                                           W >> 1, None, None), "av1r_get_output")
        return y, u, v

    def get_output_async(self, y, u, v):
        """Start the read-back of the oldest queued frame into numpy planes y, u, v (kept alive
        by the caller until waited for; av1r_get_output_async).  Returns an OutputTicket, or None
        when no frame is queued."""
        t = C.c_void_p()
        rc = self.l.av1r_get_output_async(self.c, y.ctypes.data, y.strides[0], u.ctypes.data, u.strides[0],
                                          v.ctypes.data, v.strides[0], None, None, C.byref(t))
        if rc == abi.AV1R_E_NO_OUTPUT:
            return None
        self._check(rc, "av1r_get_output_async")
        return OutputTicket(self, t, (y, u, v))

    def output_size(self):
        """(width, height) of the oldest queued frame, or None."""
        w, h = C.c_int(), C.c_int()
        if self.l.av1r_get_output(self.c, None, 0, None, 0, None, 0, C.byref(w), C.byref(h)) != 0:
            return None
        return w.value, h.value

    def read_stage(self, stage):
        W, H = self.last.frame_width, self.last.frame_height
        out = []
        for p in range(3):
            w, h = (W, H) if p == 0 else (W >> 1, H >> 1)
            a = np.empty((h, w), np.uint8)
            self._check(self.l.av1r_read_stage(self.c, stage, p, a.ctypes.data, w), "av1r_read_stage")
            out.append(a)
        return out

    def last_frame_times(self):
        t = [C.c_float() for _ in range(4)]
        self._check(self.l.av1r_last_frame_times(self.c, *[C.byref(x) for x in t]), "av1r_last_frame_times")
        return [x.value for x in t]

    def set_flow_spins(self, spins):
        """Test hook: polls before a k_flow wait gives up (0 = default; 1 forces timeouts)."""
        self._check(self.l.av1r_set_flow_spins(self.c, int(spins)), "av1r_set_flow_spins")

    def ref_release(self, slot_mask):
        """Drop the reference store's hold on the slots of `slot_mask` (av1r_ref_release)."""
        self._check(self.l.av1r_ref_release(self.c, int(slot_mask)), "av1r_ref_release")

    def set_schedule(self, mode):
        """1: dataflow kernel k_flow (default), 0: one launch per dependency level."""
        self._check(self.l.av1r_set_schedule(self.c, int(mode)), "av1r_set_schedule")

    def recon_kernel_times(self):
        """(totals_ms[k_inter, k_resid, k_flow], frames) of the frames stage_times() will report."""
        t = (C.c_float * 3)()
        n = C.c_int()
        self._check(self.l.av1r_recon_kernel_times(self.c, t, C.byref(n)), "av1r_recon_kernel_times")
        return list(t), n.value

    def stage_times(self):
        """(totals_ms[recon, lf, cdef, lr], frames) since the previous call (timing=True)."""
        t = (C.c_float * 4)()
        n = C.c_int()
        self._check(self.l.av1r_stage_times(self.c, t, C.byref(n)), "av1r_stage_times")
        return list(t), n.value

    def last_frame_stats(self):
        lv, ub = C.c_int(), C.c_uint64()
        self.l.av1r_last_frame_stats(self.c, C.byref(lv), C.byref(ub))
        return lv.value, ub.value


class OutputTicket:
    """An asynchronous frame read-back (av1r_output_query / av1r_output_wait)."""

    def __init__(self, dec, t, planes):
        self.dec, self.t, self.planes = dec, t, planes

    def ready(self):
        rc = self.dec.l.av1r_output_query(self.t)
        if rc < 0:
            self.dec._check(rc, "av1r_output_query")
        return rc == 1

    def wait(self):
        """Block until the planes have landed; returns them (the ticket is released)."""
        t, self.t = self.t, None
        if t is None:
            raise BackendError("ticket already waited for")
        self.dec._check(self.dec.l.av1r_output_wait(t), "av1r_output_wait")
        return self.planes
