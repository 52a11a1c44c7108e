"""Build and load the HIP backend library (libav1r.so, C-ABI of include/av1r.h).

The library is built in-tree for gfx950 with hipcc (no JIT cache): it is the product
path, and loading fails loudly if it is missing -- there is no CPU fallback."""
import ctypes as C
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(BUILD, "libav1r.so")
# (source, object, extra flags): recon.hip twice -- the level kernels, and k_flow alone.
# Both without machine-level loop-invariant hoisting: in k_flow's persistent loop it hoists
# ~50 constants into VGPRs for every code path (177 instead of 124 VGPRs, half the
# occupancy); k_inter at 4 waves/SIMD spills less without it (64 vs 96 B/lane; 6 % faster)
SRCS = [("recon.hip", "recon", ["-mllvm", "-disable-machine-licm"]),
        ("recon.hip", "recon_flow", ["-DAV1R_FLOW_PART", "-mllvm", "-disable-machine-licm"]),
        ("filters.hip", "filters", []),
        ("av1r_host.cpp", "av1r_host", [])]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include")]


# host-only C++ linked into the same library: the parser (include/av1p.h) and the
# whole-decoder facade (include/av1dec.h, include/YamiAv1/Av1Decoder.h)
HOST_SRCS = [("parse/obu.cpp", "p_obu"), ("parse/block.cpp", "p_block"), ("parse/api.cpp", "p_api"),
             ("app/decoder.cpp", "app_decoder"), ("app/yami.cpp", "app_yami"), ("av1r_pipeline.cpp", "av1r_pipeline")]
CLI = os.path.join(BUILD, "av1dec")
YAMI_APP = os.path.join(BUILD, "yami_decode")


def _host_cmd(src, obj):
    return [os.environ.get("CXX", "g++"), "-std=c++17", "-O2", "-fPIC", "-Wall", "-Wno-class-memaccess",
            "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc", "parse"), "-c",
            os.path.join(PKG, "csrc", src), "-o", obj]


def _stale():
    if not all(os.path.exists(p) for p in (LIB, CLI, YAMI_APP)):
        return True
    t = min(os.path.getmtime(p) for p in (LIB, CLI, YAMI_APP))
    deps = [os.path.join(PKG, "csrc", f) for f in os.listdir(os.path.join(PKG, "csrc"))]
    for sub in ("parse", "app"):
        deps += [os.path.join(PKG, "csrc", sub, f) for f in os.listdir(os.path.join(PKG, "csrc", sub))]
    for dp, _, fs in os.walk(os.path.join(ROOT, "include")):
        deps += [os.path.join(dp, f) for f in fs]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, jobs=3, out=None, defines=(), src_flags=None):
    """src_flags: {object: extra flags} replacing SRCS' own (A/B builds)."""
    """Compile every HIP/C++ source for gfx950 and link libav1r.so in-tree (or `out`, e.g.
    a -DAV1R_TRACE build for tools/trace_run.py)."""
    lib_path = out or LIB
    if out is None and not defines and not force and not _stale():
        return LIB
    os.makedirs(BUILD, exist_ok=True)
    tag = "" if out is None else "_" + os.path.splitext(os.path.basename(out))[0]
    procs, objs = [], []
    for s, name, extra in SRCS:
        src = os.path.join(PKG, "csrc", s)
        obj = os.path.join(BUILD, name + tag + ".o")
        if src_flags is not None and name in src_flags:
            extra = src_flags[name]
        cmd = [HIPCC] + FLAGS + extra + ["-D" + d for d in defines] + (["-x", "hip"] if s.endswith(".cpp") else []) \
            + ["-c", src, "-o", obj]
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
        if len(procs) >= jobs:
            if procs.pop(0).wait() != 0:
                raise RuntimeError("hipcc failed")
    for src, name in HOST_SRCS:
        obj = os.path.join(BUILD, name + tag + ".o")
        procs.append(subprocess.Popen(_host_cmd(src, obj)))
        objs.append(obj)
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    tmp = lib_path + ".tmp"
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o", tmp] + objs)
    os.replace(tmp, lib_path)
    if out is None:
        # the command-line decoder (tests/Av1Dec.cpp's counterpart), linked to this library
        tmp = CLI + ".tmp"
        subprocess.check_call([os.environ.get("CXX", "g++"), "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"),
                               "-o", tmp, os.path.join(PKG, "csrc", "app", "av1dec.cpp"), "-L" + BUILD, "-lav1r",
                               "-Wl,-rpath,$ORIGIN"])
        os.replace(tmp, CLI)
        # an application of the Yami decoder API (include/yami/yami_av1.h, createVideoDecoder)
        tmp = YAMI_APP + ".tmp"
        subprocess.check_call([os.environ.get("CXX", "g++"), "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"),
                               "-o", tmp, os.path.join(PKG, "csrc", "app", "yami_decode.cpp"), "-L" + BUILD, "-lav1r",
                               "-Wl,-rpath,$ORIGIN"])
        os.replace(tmp, YAMI_APP)
    return lib_path


PARSE_LIB = os.path.join(BUILD, "libav1p.so")
PARSE_SRCS = ("obu.cpp", "block.cpp", "api.cpp")
CXX = os.environ.get("CXX", "g++")


def build_parser(force=False, out=None, extra=()):
    """Host parser (include/av1p.h): plain C++, no device code -- libav1p.so in-tree."""
    lib_path = out or PARSE_LIB
    pdir = os.path.join(PKG, "csrc", "parse")
    if out is None and not force and not extra and os.path.exists(lib_path):
        t = os.path.getmtime(lib_path)
        deps = [os.path.join(pdir, f) for f in os.listdir(pdir)] + [os.path.join(ROOT, "include", f)
                                                                   for f in os.listdir(os.path.join(ROOT, "include"))]
        if all(os.path.getmtime(d) <= t for d in deps):
            return lib_path
    os.makedirs(BUILD, exist_ok=True)
    tmp = f"{lib_path}.{os.getpid()}.tmp"  # (concurrent test workers may build at once)
    subprocess.check_call([CXX, "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-Wno-class-memaccess",
                           "-I" + os.path.join(ROOT, "include"), "-I" + pdir, *extra, "-o", tmp]
                          + [os.path.join(pdir, s) for s in PARSE_SRCS])
    os.replace(tmp, lib_path)
    return lib_path


_plib = None


def parser_lib():
    global _plib
    if _plib is not None:
        return _plib
    path = os.environ.get("AV1P_LIB", PARSE_LIB)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run av1dec_amd.native.build_parser()")
    l = C.CDLL(path)
    vp = C.c_void_p
    l.av1p_create.argtypes = [C.POINTER(vp)]
    l.av1p_destroy.argtypes = [vp]
    l.av1p_destroy.restype = None
    l.av1p_decode_tu.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
    l.av1p_frame.argtypes = [vp, C.c_int]
    l.av1p_frame.restype = vp
    l.av1p_last_error.argtypes = [vp]
    l.av1p_last_error.restype = C.c_char_p
    l.av1p_set_tile_threads.argtypes = [vp, C.c_int]
    l.av1p_set_mode_info.argtypes = [vp, C.c_int]
    l.av1p_set_frame_generations.argtypes = [vp, C.c_int]
    _plib = l
    return l


PARSE_EXPORTS = ["av1p_create", "av1p_destroy", "av1p_decode_tu", "av1p_frame", "av1p_last_error", "av1p_set_tile_threads",
                 "av1p_set_mode_info", "av1p_set_frame_generations"]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # AV1R_LIB: an alternative build of the same library (A/B measurements)
    path = os.environ.get("AV1R_LIB", LIB)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run av1dec_amd.native.build() (hipcc, gfx950)")
    l = C.CDLL(path)
    vp, i, u8p = C.c_void_p, C.c_int, C.c_void_p
    l.av1r_create.argtypes = [i, C.POINTER(vp)]
    l.av1r_destroy.argtypes = [vp]
    l.av1r_destroy.restype = None
    l.av1r_decode_frame.argtypes = [vp, vp]
    l.av1r_frame_begin.argtypes = [vp, vp]
    l.av1r_submit_tile.argtypes = [vp, vp]
    l.av1r_frame_end.argtypes = [vp]
    l.av1r_show_existing.argtypes = [vp, i, i]
    l.av1r_output_pending.argtypes = [vp]
    l.av1r_get_output.argtypes = [vp, u8p, i, u8p, i, u8p, i, C.POINTER(i), C.POINTER(i)]
    l.av1r_read_stage.argtypes = [vp, i, i, u8p, i]
    l.av1r_synchronize.argtypes = [vp]
    l.av1r_set_timing.argtypes = [vp, i]
    l.av1r_set_keep_stages.argtypes = [vp, i]
    l.av1r_last_frame_times.argtypes = [vp] + [C.POINTER(C.c_float)] * 4
    l.av1r_last_frame_stats.argtypes = [vp, C.POINTER(i), C.POINTER(C.c_uint64)]
    l.av1r_last_error.argtypes = [vp]
    l.av1r_last_error.restype = C.c_char_p
    l.av1r_stage_times.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(i)]
    l.av1r_recon_kernel_times.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(i)]
    l.av1r_set_schedule.argtypes = [vp, i]
    l.av1r_prepare.argtypes = [vp, vp, C.POINTER(i)]
    l.av1r_decode_prepared.argtypes = [vp, i]
    l.av1r_decode_prepared_batch.argtypes = [C.POINTER(vp), C.POINTER(i), i]
    l.av1r_release_prepared.argtypes = [vp, i]
    l.av1r_set_discard_output.argtypes = [vp, i]
    l.av1r_check_batch.argtypes = [vp, C.POINTER(i), C.c_char_p, i]
    l.av1r_sizeof.argtypes = [i]
    l.av1r_sizeof.restype = C.c_size_t
    l.av1r_set_flow_spins.argtypes = [vp, C.c_uint32]
    l.av1r_flow_debug.argtypes = [C.POINTER(C.c_uint32), i, i, C.POINTER(i)]
    l.av1r_set_fast_intra.argtypes = [i]
    l.av1r_packed_data.argtypes = [vp, C.POINTER(C.c_size_t)]
    l.av1r_packed_data.restype = vp
    l.av1r_pack.argtypes = [vp, C.POINTER(vp)]
    l.av1r_packed_free.argtypes = [vp]
    l.av1r_packed_free.restype = None
    l.av1r_packed_bytes.argtypes = [vp]
    l.av1r_packed_bytes.restype = C.c_size_t
    l.av1r_pack_last_error.argtypes = []
    l.av1r_pack_last_error.restype = C.c_char_p
    l.av1r_decode_packed_batch.argtypes = [C.POINTER(vp), C.POINTER(vp), i]
    l.av1r_busy.argtypes = [vp]
    l.av1r_pack_profile.argtypes = [C.POINTER(C.c_uint64), i, i]
    l.av1r_pipeline_run.argtypes = [C.POINTER(vp), i, C.POINTER(StreamSource), C.c_int64, i, i, C.POINTER(PipelineStats)]
    l.av1r_pipeline_open.argtypes = [C.POINTER(vp), i, C.POINTER(StreamSource), i, i, C.POINTER(vp)]
    l.av1r_pipeline_step.argtypes = [vp, C.c_int64, C.POINTER(PipelineStats)]
    l.av1r_pipeline_launched.argtypes = [vp, C.POINTER(C.c_int64), i]
    l.av1r_pipeline_close.argtypes = [vp]
    l.av1r_pipeline_close.restype = None
    l.av1r_cycle_next.argtypes = [vp, i, C.POINTER(vp)]
    l.av1r_ivf_source_create.argtypes = [C.POINTER(vp), C.POINTER(C.c_size_t), i, C.POINTER(StreamSource)]
    l.av1r_ivf_source_destroy.argtypes = [C.POINTER(StreamSource)]
    l.av1r_ivf_source_destroy.restype = None
    l.av1r_get_output_async.argtypes = [vp, u8p, i, u8p, i, u8p, i, C.POINTER(i), C.POINTER(i), C.POINTER(vp)]
    l.av1r_output_query.argtypes = [vp]
    l.av1r_output_start.argtypes = [vp]
    l.av1r_output_wait.argtypes = [vp]
    l.av1r_set_output_prefetch.argtypes = [vp, i]
    l.av1r_pipeline_set_output.argtypes = [vp, C.POINTER(OutputSink)]
    l.av1r_ring_sink_create.argtypes = [i, i, i, i, C.POINTER(OutputSink)]
    l.av1r_ring_sink_destroy.argtypes = [C.POINTER(OutputSink)]
    l.av1r_ring_sink_destroy.restype = None
    l.av1r_ring_sink_delivered.argtypes = [C.POINTER(OutputSink), i]
    l.av1r_ring_sink_delivered.restype = C.c_int64
    l.av1r_ring_sink_frame.argtypes = [C.POINTER(OutputSink), i, C.c_int64, C.POINTER(i), C.POINTER(i)]
    l.av1r_ring_sink_frame.restype = vp
    l.av1r_frame_layout.argtypes = [i, i, C.POINTER(i), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    _lib = l
    return l


class StreamSource(C.Structure):  # av1r_stream_source
    _fields_ = [("next", C.c_void_p), ("user", C.c_void_p), ("stable", C.c_int), ("release", C.c_void_p)]


SINK_ACQUIRE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_int))
SINK_DELIVER = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int)


class OutputSink(C.Structure):  # av1r_output_sink
    _fields_ = [("acquire", C.c_void_p), ("deliver", C.c_void_p), ("user", C.c_void_p)]


SINK_INFLIGHT = 8  # AV1R_SINK_INFLIGHT


class PipelineStats(C.Structure):  # av1r_pipeline_stats
    _fields_ = [("frames", C.c_uint64), ("batches", C.c_uint64), ("elapsed_s", C.c_double),
                ("produce_s", C.c_double), ("pack_s", C.c_double), ("wait_s", C.c_double),
                ("launch_s", C.c_double), ("output_s", C.c_double)]


class Cycle(C.Structure):  # av1r_cycle
    _fields_ = [("batches", C.c_void_p), ("count", C.POINTER(C.c_int)), ("pos", C.POINTER(C.c_int64)),
                ("n_streams", C.c_int)]


EXPORTS = [
    "av1r_create", "av1r_destroy", "av1r_decode_frame", "av1r_frame_begin", "av1r_submit_tile",
    "av1r_frame_end", "av1r_show_existing", "av1r_output_pending", "av1r_get_output",
    "av1r_read_stage", "av1r_synchronize", "av1r_last_frame_times", "av1r_set_timing",
    "av1r_set_keep_stages", "av1r_last_frame_stats", "av1r_last_error", "av1r_sizeof",
    "av1r_check_batch", "av1r_prepare", "av1r_decode_prepared", "av1r_release_prepared",
    "av1r_set_discard_output", "av1r_stage_times", "av1r_decode_prepared_batch", "av1r_recon_kernel_times",
    "av1r_set_schedule", "av1r_set_flow_spins", "av1r_flow_debug", "av1r_pack", "av1r_packed_free",
    "av1r_packed_bytes", "av1r_pack_last_error", "av1r_decode_packed_batch", "av1r_busy", "av1r_pack_profile",
    "av1r_pipeline_run", "av1r_pipeline_open", "av1r_pipeline_step", "av1r_pipeline_launched",
    "av1r_pipeline_close", "av1r_cycle_next", "av1r_ivf_source_create", "av1r_ivf_source_destroy",
    "av1r_set_fast_intra", "av1r_packed_data",
    "av1r_get_output_async", "av1r_output_query", "av1r_output_start", "av1r_output_wait", "av1r_set_output_prefetch", "av1r_pipeline_set_output",
    "av1r_ring_sink_create", "av1r_ring_sink_destroy", "av1r_ring_sink_delivered", "av1r_ring_sink_frame",
    "av1r_frame_layout", "av1r_ref_release",
    "av1r_set_strip_levels", "av1r_set_filter_fusion", "av1r_set_flow_wave",  # (deprecated no-ops)
]


_hip = None


def hip():
    """The HIP runtime libav1r.so itself is linked to (ctypes), for the measurement helpers
    below: torch carries its own runtime, which cannot share a process with this one."""
    global _hip
    if _hip is None:
        lib()  # loads libamdhip64 as a dependency of libav1r.so
        h = C.CDLL("libamdhip64.so.7")
        vp = C.c_void_p
        h.hipHostMalloc.argtypes = [C.POINTER(vp), C.c_size_t, C.c_uint]
        h.hipHostFree.argtypes = [vp]
        h.hipMalloc.argtypes = [C.POINTER(vp), C.c_size_t]
        h.hipFree.argtypes = [vp]
        h.hipMemcpy.argtypes = [vp, vp, C.c_size_t, C.c_int]
        h.hipEventCreate.argtypes = [C.POINTER(vp)]
        h.hipEventRecord.argtypes = [vp, vp]
        h.hipEventSynchronize.argtypes = [vp]
        h.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), vp, vp]
        h.hipEventDestroy.argtypes = [vp]
        h.hipMemcpyAsync.argtypes = [vp, vp, C.c_size_t, C.c_int, vp]
        h.hipSetDevice.argtypes = [C.c_int]
        h.hipDeviceSynchronize.argtypes = []
        h.hipDeviceGetPCIBusId.argtypes = [C.c_char_p, C.c_int, C.c_int]
        _hip = h
    return _hip


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) of `n` bytes."""

    def __init__(self, n):
        self.n = n
        self.ptr = C.c_void_p()
        if hip().hipHostMalloc(C.byref(self.ptr), n, 0) != 0:
            raise MemoryError(f"hipHostMalloc({n})")

    def close(self):
        if self.ptr:
            hip().hipHostFree(self.ptr)
            self.ptr = C.c_void_p()


def copy_peak_gbps(device=0, nbytes=1 << 30, reps=10):
    """Device-to-device copy rate (read + write bytes / s, best of `reps`, HIP events)."""
    h = hip()
    h.hipSetDevice(device)
    a, b = C.c_void_p(), C.c_void_p()
    if h.hipMalloc(C.byref(a), nbytes) or h.hipMalloc(C.byref(b), nbytes):
        raise MemoryError("hipMalloc")
    e0, e1 = C.c_void_p(), C.c_void_p()
    h.hipEventCreate(C.byref(e0))
    h.hipEventCreate(C.byref(e1))
    try:
        h.hipMemcpyAsync(b, a, nbytes, 3, None)  # hipMemcpyDeviceToDevice
        h.hipDeviceSynchronize()
        best = None
        for _ in range(reps):
            h.hipEventRecord(e0, None)
            h.hipMemcpyAsync(b, a, nbytes, 3, None)
            h.hipEventRecord(e1, None)
            h.hipEventSynchronize(e1)
            ms = C.c_float()
            h.hipEventElapsedTime(C.byref(ms), e0, e1)
            best = ms.value if best is None else min(best, ms.value)
    finally:
        h.hipEventDestroy(e0)
        h.hipEventDestroy(e1)
        h.hipFree(a)
        h.hipFree(b)
    return 2 * nbytes / (best * 1e-3) / 1e9

