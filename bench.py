#!/usr/bin/env python3
"""bench.py -- frames/s of the MI355X AV1 reconstruction + in-loop filter backend.

Workload (BASELINE.json configs[2] streams, batched as configs[4]): S = 8 independent
synthetic 1920x1080 8-bit 4:2:0 streams per GPU -- the per-GPU share of the 64-stream
batch over 8 GPUs -- each 1 key + 59 inter frames (tools/synth: 8-tap subpel, compound
avg/dist/wedge/diff-weighted, inter-intra, OBMC, local warp, LF + CDEF + LR), cycled, stream
j offset by j*F/S frames so every window of steps holds its share of key frames.  One step
= one frame of every stream through recon -> deblock -> CDEF -> loop restoration in shared
launches.

value (headline): the host-inclusive rate.  The frame batches (tools/synth's output, the
same av1r_frame_batch records the host parser emits, checked against the pinned oracle) sit
in host memory; inside the timed region every frame is validated, scheduled and packed
by worker threads (av1r_pack) up to 3 steps ahead, uploaded over PCIe and decoded
(av1r_decode_packed_batch).  Reported beside it: device_only_fps (batches already
scheduled and resident in HBM, av1r_prepare), one stream alone, the per-frame streaming
API from one thread and from one thread per stream.

Multi-GPU (--gpus N: started as N rank processes by this script itself, or by
torch.distributed.run, which sets WORLD_SIZE): every rank decodes its own
streams on its own GPU -- streams shard over GPUs with no data-path collective (SURVEY.md
8e); a gloo barrier brackets the timed region and the MAX elapsed over ranks is used.
value = N * S * steps / max_elapsed ("weak" scaling).

Also reported: roofline of the dominant stage (algorithmic bytes / device time, vs the
8 TB/s HBM3E peak) and the CPU baseline (the C oracle -- a restatement of the
reference's algorithm -- on a bounded sample of stream 0, 1 core).
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (width, height, tiles, seed)
    "1080p": (1920, 1080, (1, 1), 0x5EED1000),
    "4k": (3840, 2160, (4, 2), 0x5EED2000),
}


def stage_bytes(frame):
    """Algorithmic HBM bytes of each stage for one frame: every stage reads
    its input planes once and writes its output once; recon also reads the reference
    pixels its inter predictions use and the batch (coefficients + metadata)."""
    from av1dec_amd import abi
    h = frame.hdr
    F = h.frame_width * h.frame_height * 3 // 2
    blocks = np.frombuffer(frame.sec["blocks"].tobytes(), abi.BLOCK_DTYPE)
    mi = np.frombuffer(frame.sec["mi"].tobytes(), abi.MI_DTYPE).reshape(h.mi_rows_alloc, h.mi_stride)
    inter = (blocks["flags"] & 1) != 0
    bw = np.array([1, 1, 2, 2, 2, 4, 4, 4, 8, 8, 8, 16, 16, 16, 32, 32, 1, 4, 2, 8, 4, 16])[blocks["mi_size"]] * 4
    bh = np.array([1, 2, 1, 2, 4, 2, 4, 8, 4, 8, 16, 8, 16, 32, 16, 32, 4, 1, 8, 2, 16, 4])[blocks["mi_size"]] * 4
    nref = 1 + (mi["ref_frame"][blocks["mi_row"], blocks["mi_col"], 1] > 0)
    ref_bytes = int(np.sum((bw * bh * nref * 3 // 2)[inter]))
    batch = frame.payload_bytes()
    return {
        "recon": F + ref_bytes + batch,
        "lf": 2 * F if (h.lf_level[0] or h.lf_level[1]) else 0,
        "cdef": 2 * F,
        "lr": (2 * F + F // 16) if h.uses_lr else 0,
    }


def stream_seed(config_seed, rank):
    """Stream i -> GPU i: every rank decodes its own independent stream."""
    return config_seed + rank


def rank_stream_ids(rank, S):
    """The global stream ids rank `rank` decodes (S per GPU, contiguous): stream i of the job
    is synthetic seed stream_seed(config_seed, i) -- disjoint shards, no data-path exchange."""
    return [rank * S + j for j in range(S)]


def rank_streams(config, rank, S, frames, width=None, height=None):
    """Rank `rank`'s shard: its S synthetic streams (frame batches), as the bench decodes them."""
    import pysynth
    W, H, tiles, seed = CONFIGS[config]
    W, H = width or W, height or H
    return [pysynth.stream(W, H, frames, stream_seed(seed, i), sb128=True, tiles=tiles) for i in rank_stream_ids(rank, S)]


def max_over_ranks(elapsed, dist=None):
    """The timed region's MAX over ranks (barrier after, so no rank races ahead)."""
    if dist is None:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    return float(t.item())


def aggregate_fps(world, steps, elapsed):
    """Whole-job frames/s: every rank decodes `steps` frames of its own stream."""
    return world * steps / elapsed


def gop_offsets(S, F):
    """Stream j starts j*F/S frames into its GOP: independent streams are not in phase, so
    any window of steps holds its share of key frames (S/F per step)."""
    return [j * F // S for j in range(S)]


class StreamScheduler:
    """S independent streams, each cycling its own F-frame GOP from its own phase (stream j
    starts j*F/S frames in), decoded in shared launches.  Each round batches the next frame
    of every stream that is ready: a stream whose key frame is still running alone on its
    own HIP stream (av1r_busy: the library launches deep frames solo so that they overlap
    the batches) sits out until it is done.  A stream always decodes its frames in order
    from its key frame (frame 0 refreshes every slot, so cycling the GOP is a valid stream).

    packed: the host-inclusive pipeline -- worker threads validate, schedule and pack
    (av1r_pack) each stream's next `depth` frames while the GPU decodes, and every round
    uploads and decodes the packed frames (av1r_decode_packed_batch); the frame batches
    (tools/synth's av1r_frame_batch records) sit in host memory.  Otherwise frames come from
    per-stream lists of prepared handles (av1r_prepare: scheduled and resident in HBM)."""

    def __init__(self, decs, F, streams=None, handles=None, workers=1, depth=3):
        from concurrent.futures import ThreadPoolExecutor
        self.decs, self.F, self.streams, self.handles, self.depth = decs, F, streams, handles, depth
        self.packed = handles is None
        self.ex = ThreadPoolExecutor(max(1, workers)) if self.packed else None
        self.pos = [0] * len(decs)
        self.q = [[] for _ in decs]  # packed: per stream, futures of its next frames
        # host profile of the packed pipeline: worker seconds in av1r_pack, launching-thread
        # seconds waiting for packed frames and inside av1r_decode_packed_batch
        self.prof = {"pack_s": 0.0, "packs": 0, "wait_s": 0.0, "launch_s": 0.0, "launches": 0}
        self._plock = __import__("threading").Lock()

    def _pack(self, frame):
        from av1dec_amd import Decoder
        t = time.perf_counter()
        p = Decoder.pack(frame)
        dt = time.perf_counter() - t
        with self._plock:
            self.prof["pack_s"] += dt
            self.prof["packs"] += 1
        return p

    def reset_prof(self):
        for k in self.prof:
            self.prof[k] = 0 if k in ("packs", "launches") else 0.0

    def _item(self, j):
        from av1dec_amd import Decoder
        if not self.packed:
            return self.handles[j][self.pos[j] % self.F]
        while len(self.q[j]) < self.depth:
            t = (self.pos[j] + len(self.q[j])) % self.F
            self.q[j].append(self.ex.submit(self._pack, self.streams[j][t]))
        t0 = time.perf_counter()
        r = self.q[j].pop(0).result()
        self.prof["wait_s"] += time.perf_counter() - t0
        return r

    def _launch(self, js):
        from av1dec_amd import Decoder
        items = [self._item(j) for j in js]
        decs = [self.decs[j] for j in js]
        if self.packed:
            t0 = time.perf_counter()
            Decoder.decode_packed_batch(decs, items)
            self.prof["launch_s"] += time.perf_counter() - t0
            self.prof["launches"] += 1
            for p in items:
                Decoder.free_packed(p)
            for j in js:  # keep the packers `depth` frames ahead
                self._top_up(j)
        else:
            Decoder.decode_prepared_batch(decs, items)
        out = [(j, self.pos[j] % self.F) for j in js]
        for j in js:
            self.pos[j] += 1
        return out

    def _top_up(self, j):
        from av1dec_amd import Decoder
        while len(self.q[j]) < self.depth:
            t = (self.pos[j] + 1 + len(self.q[j])) % self.F
            self.q[j].append(self.ex.submit(self._pack, self.streams[j][t]))

    def stagger(self):
        """Bring stream j alone to frame j*F/S (untimed setup)."""
        for j, off in enumerate(gop_offsets(len(self.decs), self.F)):
            while self.pos[j] < off:
                self._launch([j])

    def run(self, k):
        """Decode the next k frames of every stream; returns the (stream, frame) pairs."""
        target = [p + k for p in self.pos]
        done = []
        while True:
            left = [j for j in range(len(self.decs)) if self.pos[j] < target[j]]
            if not left:
                return done
            ready = [j for j in left if not self.decs[j].busy()]
            if not ready:
                time.sleep(50e-6)
                continue
            done += self._launch(ready)

    def close(self):
        from av1dec_amd import Decoder
        if self.ex:
            for q in self.q:
                for f in q:
                    Decoder.free_packed(f.result())
            self.q = [[] for _ in self.decs]
            self.ex.shutdown()


def ivf_streams(rank, S, frames, name="1080p_s1", seed=0x5EED1000):
    """Rank `rank`'s shard of configs[4] as real bitstreams: S synthetic 1080p IVF streams from
    the bitstream writer (tools/bsw, configuration 1080p_s1; stream i of the job has seed
    0x5EED1000 + i, so stream 0 is the one tests/golden/bsw.json pins to the reference's MD5),
    written in parallel (untimed).  (configs[3]: name 4k_s2_tiles4x2, seed 0x5EED2000.)"""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "tools", "bsw"))
    import pybsw
    ids = rank_stream_ids(rank, S)
    with ThreadPoolExecutor(min(S, 16)) as ex:
        return list(ex.map(lambda i: pybsw.stream_ivf(name, seed=seed + i, frames=frames), ids))


def ivf_leg(decs, streams, frames, size="1920x1080", name="1080p_s1", seed=0x5EED1000):
    """configs[4] end to end: every stream's IVF parsed on its own host thread and packed
    while the GPU decodes, one frame of every ready stream per shared launch
    (av1dec_amd.pipeline.IvfPipeline); one untimed pass, then a timed one.  Multi-tile
    frames (configs[3]) are parsed tile-parallel (av1p_set_tile_threads)."""
    from av1dec_amd.pipeline import run_native
    # two workers per stream: a stream's next frame parses while its previous one packs (the
    # IVF source keeps two parsed units alive, av1r_pipeline.cpp).  Against one worker per
    # stream: 1080p 365-382 vs 352-357 frames/s, 4K 4x2 tiles 97-101 vs 75-77
    # (profiles/r05_ab_ivf_workers2.txt; with the slower parser of r05_ab_ivf_workers.txt the
    # 1080p leg had measured no faster)
    per = int(os.environ.get("AV1R_BENCH_IVF_WORKERS_PER_STREAM", "2"))  # (A/B)
    workers = per * len(streams)
    run_native(decs, "ivf", streams, workers=workers)
    t0 = time.perf_counter()
    st = run_native(decs, "ivf", streams, workers=workers)
    dt = time.perf_counter() - t0
    n = int(st["frames"])
    return {"fps": round(n / dt, 3), "streams": len(streams), "frames_per_stream": frames,
            "frames": n, "elapsed_s": round(dt, 3),
            "parse_ms_per_frame": round(1e3 * st["produce_s"] / n, 3),
            "pack_ms_per_frame": round(1e3 * st["pack_s"] / n, 3),
            "stream_bytes_per_frame": int(sum(len(s) for s in streams) / n),
            "batches": int(st["batches"]), "host_workers": workers,
            "workload": f"{len(streams)} synthetic {size} IVF streams from tools/bsw ({name}: 1 key + "
                        f"{frames - 1} inter, seeds {seed:#x}+stream), parsed by the host parser (one frame of a stream at a "
                        f"time) and packed by {workers} native workers (av1r_pipeline_run: a stream's next frame "
                        f"parses while its previous one packs), decoded in shared launches; parse inside the timed "
                        f"region"}


_RANK_CPUS = None  # this rank's CPU set once bind_rank_cpus has bound it (N > 1)


def host_workers():
    """Packing threads: the box's CPU share (OMP_NUM_THREADS is set to it there) less the
    launching thread (AV1R_BENCH_WORKERS overrides, A/B).  A rank bound to its own CPUs
    (bind_rank_cpus, N > 1) takes its share of them: the node's CPUs divided by the ranks
    on that node."""
    if os.environ.get("AV1R_BENCH_WORKERS"):
        return int(os.environ["AV1R_BENCH_WORKERS"])
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    if _RANK_CPUS is not None:
        share = len(_RANK_CPUS)
    return max(1, min(share, 32) - 1)


def parse_cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (sysfs cpulist format)."""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_node(local):
    """NUMA node of GPU `local`, read without starting the HIP runtime (whose threads would
    keep the full CPU mask when the rank binds itself afterwards): the KFD topology's GPU
    nodes in enumeration order (the order the runtime numbers devices in, filtered by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES), the node's PCI location, then sysfs
    (/sys/bus/pci/devices/<bdf>/numa_node); -1 when unknown."""
    try:
        base = "/sys/class/kfd/kfd/topology/nodes"
        gpus = []
        for n in sorted((d for d in os.listdir(base) if d.isdigit()), key=int):
            with open(f"{base}/{n}/properties") as f:
                props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
            if int(props.get("simd_count", "0")) > 0:
                gpus.append(props)
        for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
            vis = os.environ.get(var, "")
            if vis and all(v.strip().isdigit() for v in vis.split(",")):
                gpus = [gpus[int(v)] for v in vis.split(",")]
        p = gpus[int(local)]
        loc, dom = int(p["location_id"]), int(p.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7}"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            return int(f.read().strip())
    except (OSError, ValueError, IndexError, KeyError):
        return -1


def split_rank_cpus(allowed, nodes, rank, node_cpus):
    """This rank's CPUs: the allowed CPUs of its GPU's NUMA node (all allowed CPUs when the
    node is unknown or none of its CPUs is allowed), divided evenly among the ranks whose GPUs
    sit on that node.  nodes: every rank's node; node_cpus(n) -> the CPUs of node n."""
    node = nodes[rank]
    pool = sorted(allowed)
    if node >= 0:
        local = [c for c in pool if c in set(node_cpus(node))]
        pool = local or pool
    peers = [r for r in range(len(nodes)) if nodes[r] == node]
    k, i = len(peers), peers.index(rank)
    chunk = pool[i * len(pool) // k:(i + 1) * len(pool) // k]
    return chunk or [pool[i % len(pool)]]


def bind_rank_cpus(rank, world, local, dist, probe_gpu=True):
    """host threads near the GPU's NUMA node, one rank's threads apart from the
    others'.  Rank r binds itself (and every thread it starts later: the native pipeline's
    packing and parse threads inherit the affinity) to its share of GPU r's node
    (split_rank_cpus), so 8 ranks of packers do not contend for the same cores.  N = 1 keeps
    the process's affinity (AV1R_BIND=1 binds it too)."""
    global _RANK_CPUS
    if world <= 1 and os.environ.get("AV1R_BIND", "0") == "0":
        return None
    node = gpu_numa_node(local) if probe_gpu else -1
    nodes = [node]
    if dist:
        nodes = [None] * world
        dist.all_gather_object(nodes, node)

    def node_cpus(n):
        try:
            return parse_cpulist(open(f"/sys/devices/system/node/node{n}/cpulist").read())
        except OSError:
            return []
    cpus = split_rank_cpus(os.sched_getaffinity(0), nodes, rank if dist else 0, node_cpus)
    os.sched_setaffinity(0, cpus)
    _RANK_CPUS = cpus
    return {"numa_node": node, "cpus": cpus}


def copy_peak_gbps(local):
    """The device's measured copy rate (report the roofline fraction against
    it as well as against the 8 TB/s spec): a 1 GiB device-to-device hipMemcpy, read +
    write bytes per second, best of 10 (av1dec_amd.native.copy_peak_gbps)."""
    from av1dec_amd import native
    return native.copy_peak_gbps(local)


def output_leg(decs, streams, pos, steps, workers):
    """The drop-in's frame delivery (Decoder::getOutput, Av1Decoder.cpp:203-211, drained after
    every unit as tests/Av1Dec.cpp:216-220 does): the headline pipeline (kept open; priming
    with one GOP untimed) with every shown frame delivered into pinned host buffers -- each
    frame's read-back starts on its context's read-back stream as soon as its batch is launched
    and lands while the next batches decode (av1r_pipeline_set_output + av1r_ring_sink, i.e.
    av1r_get_output_async / av1r_output_query).  fps = frames whose bytes have landed in host
    memory / the step's time (every frame of the step is delivered before it returns).  The
    streams continue from `pos` (their GOP phases staggered as in the headline); `pos` is
    advanced to where they stop."""
    from av1dec_amd.pipeline import NativePipeline, RingSink
    for d in decs:
        d.set_discard_output(False)
    W, H = streams[0][0].hdr.frame_width, streams[0][0].hdr.frame_height
    F = len(streams[0])
    sink = RingSink(len(decs), W, H)
    pl = NativePipeline(decs, streams, pos, depth=0, workers=workers)
    try:
        pl.set_output(sink)
        pl.step(F)  # priming, untimed: the workers reach their look-ahead
        n0 = sink.delivered()
        t0 = time.perf_counter()
        st = pl.step(steps)
        dt = time.perf_counter() - t0
        k = sink.delivered() - n0
        pl.set_output(None)
        pos[:] = pl.positions()
    finally:
        pl.close()
        sink.close()
        for d in decs:
            d.set_discard_output(True)
    return {"fps": round(k / dt, 3), "frames": k, "decoded": int(st["frames"]), "elapsed_s": round(dt, 4),
            "delivered_GBps": round(k * W * H * 1.5 / dt / 1e9, 2),
            "launcher_idle_ms_per_step": round(1e3 * st["wait_s"] / max(steps, 1), 3),
            "launcher_submit_ms_per_step": round(1e3 * st["launch_s"] / max(steps, 1), 3),
            "launcher_output_ms_per_step": round(1e3 * st["output_s"] / max(steps, 1), 3),
            "pack_ms_per_frame": round(1e3 * st["pack_s"] / max(st["frames"], 1), 3), "batches": int(st["batches"]),
            "method": "native pipeline kept open, every shown frame read back asynchronously into pinned host "
                      "buffers while later batches decode (av1r_pipeline_set_output + av1r_ring_sink); "
                      "one GOP of priming untimed"}


def cpu_model():
    try:
        return next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        return "unknown"


def cpu_baseline(frames, budget_s):
    """The C oracle (reference algorithm restated, single-threaded) on the first frames."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    o = pyoracle.Oracle(keep_stages=False)
    n = 0
    t0 = time.perf_counter()
    while n < len(frames):
        o.decode_frame(frames[n])
        while o.output_pending():
            o.get_output()
        n += 1
        if time.perf_counter() - t0 > budget_s and n >= 2:
            break
    dt = time.perf_counter() - t0
    o.close()
    return n / dt, n, dt


def box_k(nframes=6):
    """k on THIS host's CPU (the committed k was measured on the build
    container's CPU): the reference decoder (oracle/_ref/av1dec_ref, built in the build
    container from the reference's own sources by oracle/Makefile -- a CPU program, shipped
    with the tree) on the writer's 1080p_s1 stream, and the oracle on the same frames parsed
    by the host parser; 1 thread each (tools/calibrate_k_1080p.py's method).  None when the
    reference binary is absent."""
    ref = os.path.join(ROOT, "oracle", "_ref", "av1dec_ref")
    if not os.path.exists(ref):
        return None
    import re
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools", "bsw"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pybsw
    import pyoracle
    from av1dec_amd import parser
    data = pybsw.stream_ivf("1080p_s1", frames=nframes, seed=0x5EED1000)
    with tempfile.NamedTemporaryFile(suffix=".ivf") as f:
        f.write(data)
        f.flush()
        out = subprocess.run([ref, "-i", f.name], capture_output=True, text=True, timeout=300).stdout
    rfps = float(re.findall(r"decode fps = ([0-9.]+)", out)[-1])
    frames = parser.Parser().decode_ivf(data)
    o = pyoracle.Oracle(keep_stages=False)
    t = time.perf_counter()
    for fr in frames:
        o.decode_frame(fr)
        while o.output_pending():
            o.get_output()
    ofps = len(frames) / (time.perf_counter() - t)
    o.close()
    return {"k": round(rfps / ofps, 4), "reference_fps": round(rfps, 4), "oracle_fps": round(ofps, 4),
            "frames": nframes, "stream": f"tools/bsw 1080p_s1 seed 0x5eed1000, {nframes} frames (1 key + {nframes - 1} inter)"}


def load_traffic(path, config, S, stage):
    """PMC-derived HBM bytes per frame of `stage` (tools/pmc_traffic.py output) if the file
    was measured on this configuration, and which measurement (commit) it is."""
    if not os.path.exists(path):
        return None, None
    try:
        tj = json.load(open(path))
        if tj.get("config") == config and tj.get("streams", 1) == S and stage in tj.get("stages", {}):
            return tj["stages"][stage], {"file": os.path.relpath(path, ROOT), "git_head": tj.get("git_head")}
    except Exception:
        pass
    return None, None


def measure(config, decs, streams, steps, warmup, workers, depth, dist, world, prime_s=2.0, prime_steps=None):
    """One configuration's rates on this rank's streams: the host-inclusive pipeline (the
    headline), the device-only rate, and the per-stage device time with the roofline of the
    dominant stage.  Returns (result dict, the StreamScheduler over prepared handles, the
    handles, the pipeline positions after the timed run)."""
    from av1dec_amd.pipeline import run_native
    S, F = len(decs), len(streams[0])

    def sync():
        for d in decs:
            d.synchronize()

    # ---- headline: the host-inclusive pipeline (per-frame validation, scheduling, packing
    # and PCIe upload of the synthetic batches inside the timed region, overlapped with the
    # GPU).  Setup (untimed): stream j brought to its own GOP phase, a priming pass of
    # ~prime_s (or exactly prime_steps GOPs: a fixed amount of work, so that separate
    # profiling passes run the same launches), then the warmup steps.  (av1r_pipeline_run: producer threads pack each
    # stream's frames ahead, the calling thread launches one frame of every ready stream per
    # batch)
    pp = StreamScheduler(decs, F, streams=streams, workers=1)
    pp.stagger()
    pp.close()
    sync()
    pos = list(pp.pos)
    # one pipeline for the priming pass, the warmup and the timed window: its packing
    # workers run continuously, `depth` frames ahead of every stream, so the window holds a
    # running decoder's steady-state work (every frame it launches was packed by the same
    # workers, which meanwhile pack the frames after the window) rather than a cold start
    # and a drain (av1r_pipeline_open / _step, include/av1r.h)
    from av1dec_amd.pipeline import NativePipeline
    pl = NativePipeline(decs, streams, pos, depth=depth, workers=workers)
    try:
        if prime_steps is not None:
            for _ in range(prime_steps):
                pl.step(F)
        else:
            t_prime = time.perf_counter()
            while time.perf_counter() - t_prime < prime_s:
                pl.step(F)
        pl.step(warmup)
        if dist:
            dist.barrier()
        pos0 = pl.positions()
        t0 = time.perf_counter()
        pr = pl.step(steps)  # synchronizes every context
        elapsed = max_over_ranks(time.perf_counter() - t0, dist)
        pos = pl.positions()
    finally:
        pl.close()
    fps = aggregate_fps(world, steps * S, elapsed)
    timed = [(j, t % F) for j in range(S) for t in range(pos0[j], pos0[j] + steps)]
    n_key = sum(1 for j, t in timed if streams[j][t].hdr.frame_type == 0)
    from av1dec_amd import Decoder, native
    lib = native.lib()
    sizes = []
    for fr in streams[0][1:9]:  # the packed batch of an inter frame (untimed)
        pk = Decoder.pack(fr)
        sizes.append(lib.av1r_packed_bytes(pk))
        Decoder.free_packed(pk)
    host_profile = {  # where the host-inclusive pipeline spends its time (rank 0)
        "packed_MB_per_inter_frame": round(sum(sizes) / max(len(sizes), 1) / 1e6, 3),
        "packing_threads": workers,
        "pack_ms_per_frame": round(1e3 * pr["pack_s"] / max(pr["frames"], 1), 3),
        "producer_utilisation": round(pr["pack_s"] / (workers * elapsed), 3),
        "launcher_idle_ms_per_step": round(1e3 * pr["wait_s"] / max(steps, 1), 3),
        "launcher_submit_ms_per_step": round(1e3 * pr["launch_s"] / max(steps, 1), 3),
        "batches": int(pr["batches"]),
    }

    # ---- device-only rate: the same streams with every batch already validated, scheduled
    # and resident in HBM (av1r_prepare), the same staggered GOP phases
    handles = [[d.prepare(f) for f in fr] for d, fr in zip(decs, streams)]
    ss = StreamScheduler(decs, F, handles=handles)
    ss.stagger()
    ss.run(F + warmup)
    sync()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ss.run(steps)
    sync()
    elapsed_dev = max_over_ranks(time.perf_counter() - t0, dist)
    device_fps = aggregate_fps(world, steps * S, elapsed_dev)

    # per-stage device time over the same batches (HIP events on the launch stream)
    for d in decs:  # every context records the launches it leads (batches and solo frames)
        d.l.av1r_set_timing(d.c, 1)
    timed2 = ss.run(steps)
    sync()
    ktot, totals, nfr = [0.0] * 3, [0.0] * 4, 0
    for d in decs:
        kt, _ = d.recon_kernel_times()
        st, nf = d.stage_times()
        ktot = [a + b for a, b in zip(ktot, kt)]
        totals = [a + b for a, b in zip(totals, st)]
        nfr += nf
        d.l.av1r_set_timing(d.c, 0)
    names = ["recon", "lf", "cdef", "lr"]
    per_frame_ms = {n: totals[k] / max(nfr, 1) for k, n in enumerate(names)}
    sb = {n: 0.0 for n in names}
    for j, t in timed2:
        for n, v in stage_bytes(streams[j][t]).items():
            sb[n] += v / len(timed2)
    dominant = max(names, key=lambda n: per_frame_ms[n])
    achieved = sb[dominant] / (per_frame_ms[dominant] * 1e-3) / 1e9
    res = {"fps": fps, "elapsed": elapsed, "n_key": n_key, "host_profile": host_profile, "device_fps": device_fps,
           "per_frame_ms": per_frame_ms, "stage_bytes": sb, "dominant": dominant, "achieved": achieved,
           "kernel_ms": {n: v / max(nfr, 1) for n, v in zip(("k_inter", "k_resid", "k_flow"), ktot)},
           "stage_GBps": {n: sb[n] / max(per_frame_ms[n], 1e-9) / 1e6 for n in names}}
    return res, ss, handles, pos


def key_frame_ms(dec, handle, reps=3):
    """Device time (recon stage, k_flow dominated) of one key frame alone on the
    chip, median of `reps`: the deep frames the batched pipeline launches solo.  (Decoding a
    key frame resets the stream's references: run it last.)"""
    dec.l.av1r_set_timing(dec.c, 1)
    t = []
    for _ in range(reps):
        dec.decode_prepared(handle)
        dec.synchronize()
        t.append(dec.last_frame_times())
    dec.l.av1r_set_timing(dec.c, 0)
    t.sort(key=lambda x: x[0])
    m = t[len(t) // 2]
    return {"recon": round(m[0], 4), "lf": round(m[1], 4), "cdef": round(m[2], 4), "lr": round(m[3], 4)}


def leg_4k(local, rank, world, dist, workers, S=2, F=30, steps=12, warmup=3, traffic=None, ivf_frames=8,
           prime_steps=None):
    """BASELINE configs[3]: S synthetic 3840x2160 streams with the 4x2 tile grid per GPU,
    host-inclusive and device-only, with its own per-stage times, roofline and PMC traffic."""
    from concurrent.futures import ThreadPoolExecutor
    import pysynth
    from av1dec_amd import Decoder
    W, H, tiles, seed = CONFIGS["4k"]
    with ThreadPoolExecutor(S) as ex:
        streams = list(ex.map(lambda i: pysynth.stream(W, H, F, stream_seed(seed, i), sb128=True, tiles=tiles),
                              rank_stream_ids(rank, S)))
    decs = [Decoder(local, keep_stages=False, timing=False) for _ in range(S)]
    for d in decs:
        d.set_discard_output(True)
    r, ss, handles, _ = measure("4k", decs, streams, steps, warmup, workers, 0, dist, world, prime_s=0.5,
                                prime_steps=prime_steps)
    kf = key_frame_ms(decs[0], handles[0][0], reps=2)
    tr, tsrc = load_traffic(traffic, "4k", S, r["dominant"]) if traffic else (None, None)
    for d, hs in zip(decs, handles):
        for hd in hs:
            d.release_prepared(hd)
    # end to end from 4x2-tile IVF bitstreams: the tiles of a frame parsed concurrently
    ivf = None
    if ivf_frames > 0:
        ivf = ivf_leg(decs, ivf_streams(rank, S, ivf_frames, "4k_s2_tiles4x2", 0x5EED2000), ivf_frames,
                      f"{W}x{H} 4x2-tile", "4k_s2_tiles4x2", 0x5EED2000)
        if dist:
            ivf["fps_all_ranks"] = round(world * ivf["frames"] / max_over_ranks(ivf["elapsed_s"], dist), 3)
    for d in decs:
        d.close()
    return {"fps": round(r["fps"], 3), "device_only_fps": round(r["device_fps"], 3), "streams_per_gpu": S,
            "steps": steps, "warmup": warmup, "ms_per_step": round(r["elapsed"] * 1e3 / steps, 4),
            "timed_key_frames": r["n_key"],
            "workload": f"{S} synthetic {W}x{H} 8-bit 4:2:0 streams per GPU, {tiles[0]}x{tiles[1]} tiles, each {F} "
                        f"frames (1 key + {F - 1} inter) cycled, seeds {seed:#x}+stream; host-inclusive as the headline",
            "roofline": {"bound": "hbm", "kernel": r["dominant"], "achieved": round(r["achieved"], 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(r["achieved"] / HBM_PEAK_GBPS, 5), "traffic": tr, "traffic_source": tsrc,
                         "bytes_per_frame": int(r["stage_bytes"][r["dominant"]]),
                         "ms_per_frame": round(r["per_frame_ms"][r["dominant"]], 4)},
            "stage_ms_per_frame": {n: round(v, 4) for n, v in r["per_frame_ms"].items()},
            "recon_kernel_ms_per_frame": {n: round(v, 4) for n, v in r["kernel_ms"].items()},
            "key_frame_alone_ms": kf,
            "host_profile": r["host_profile"],
            "ivf_end_to_end": ivf}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` from a plain shell: start N rank processes of this script (rank r on
    GPU r, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them)
    and wait for them.  The parent never touches the GPU (no HIP call before or after the
    children start, and no exec: the children are child processes); rank 0 prints the line.
    If a rank fails the others are stopped, and the worst exit status is returned.  The unit
    each rank replicates is the reference's single-stream decode loop (tests/Av1Dec.cpp:199-224),
    over its own disjoint shard of the streams."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0:
                    rc = rc or c
                    for q in live:  # a lost rank would leave the others waiting at a barrier
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return rc if rc >= 0 else 128 - rc


def dry_run(args, rank, world, dist):
    """--dry-run: the N-rank plumbing without a GPU (CPU tests): every rank builds its own
    shard exactly as the real run does (rank_streams, at 64x64 so it takes milliseconds),
    times it through the same barrier + MAX-over-ranks, and rank 0 prints the line with every
    rank's stream ids and a digest of its shard's batches (gathered for the report only)."""
    import hashlib
    S = max(1, args.streams)
    bound = bind_rank_cpus(rank, world, int(os.environ.get("LOCAL_RANK", "0")), dist, probe_gpu=False)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    streams = rank_streams(args.config, rank, S, 2, width=64, height=64)
    h = hashlib.md5()
    for fr in streams:
        for f in fr:
            h.update(f.to_bytes())
    elapsed = max_over_ranks(time.perf_counter() - t0, dist)
    mine = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "pid": os.getpid(),
            "stream_ids": rank_stream_ids(rank, S), "digest": h.hexdigest(),
            "cpus": bound["cpus"] if bound else sorted(os.sched_getaffinity(0)), "host_workers": host_workers()}
    shards = [mine]
    if dist:
        shards = [None] * world
        dist.all_gather_object(shards, mine)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "elapsed": elapsed,
                          "value": aggregate_fps(world, 2 * S, elapsed), "shards": shards,
                          "config": {"parallelism": f"stream-per-GPU x{world}", "streams_per_gpu": S}}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60, help="timed batch steps (one frame of every stream each)")
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--config", default="1080p", choices=sorted(CONFIGS))
    ap.add_argument("--streams", type=int, default=8,
                    help="independent streams per GPU, decoded in shared launches (configs[4]: 64 streams / 8 GPUs)")
    ap.add_argument("--frames", type=int, default=60, help="stream length (1 key + inter)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ivf-frames", type=int, default=24, help="frames per stream of the IVF end-to-end leg (0: skip)")
    ap.add_argument("--no-4k", action="store_true", help="skip the configs[3] 4K leg of a 1080p run")
    ap.add_argument("--output-steps", type=int, default=180, help="steps of the frame-delivery leg (0: skip)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per frame (tools/pmc_traffic.py)")
    ap.add_argument("--traffic-4k", default=os.path.join(ROOT, "profiles", "traffic_4k.json"))
    ap.add_argument("--prime-steps", type=int, default=None,
                    help="priming GOPs of the headline pipeline (default: ~2 s of them); a fixed count gives "
                         "every rocprofv3 --pmc pass the same work (tools/gpu_evidence_r05.sh)")
    ap.add_argument("--dry-run", action="store_true",
                    help="the N-rank launch and sharding only, no GPU (tests/test_multi.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `bench.py --gpus N`: one process per GPU, started here before anything
        # touches a GPU (torch.distributed.run sets WORLD_SIZE itself and lands below)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")
    if args.dry_run:
        dry_run(args, rank, world, dist)
        if dist:
            dist.destroy_process_group()
        return

    # before any thread of ours (or of the HIP runtime) starts: the rank's share of its GPU's
    # NUMA node, found from sysfs
    bound = bind_rank_cpus(rank, world, local, dist)
    from av1dec_amd import Decoder, native

    native.lib()
    W, H, tiles, seed = CONFIGS[args.config]
    S = max(1, args.streams)
    F = args.frames
    # stream i of the job = rank * S + j (independent streams, one GPU each)
    streams = rank_streams(args.config, rank, S, F)
    decs = [Decoder(local, keep_stages=False, timing=False) for _ in range(S)]
    for d in decs:
        d.set_discard_output(True)
    workers = host_workers()
    # frames packed ahead per stream (AV1R_BENCH_DEPTH; 0: the pipeline's default,
    # max(8, 2 * ceil(workers / streams)) -- 8 at 1080p x 8 streams, 16 at 4K x 2)
    depth = int(os.environ.get("AV1R_BENCH_DEPTH", "0"))
    depth_eff = depth if depth > 0 else max(8, 2 * -(-max(1, workers) // len(streams)))

    def sync():
        for d in decs:
            d.synchronize()

    r, ss, handles, pos = measure(args.config, decs, streams, args.steps, args.warmup, workers, depth, dist, world,
                                  prime_steps=args.prime_steps)
    fps, elapsed = r["fps"], r["elapsed"]
    dominant, achieved, per_frame_ms, sb = r["dominant"], r["achieved"], r["per_frame_ms"], r["stage_bytes"]
    traffic, traffic_src = load_traffic(args.traffic, args.config, S, dominant)
    lead = decs[0]

    # ---- frame delivery: the headline pipeline with every frame read back to host memory,
    # asynchronously (the streams continue where the device-only leg left them, staggered)
    out_pos = list(ss.pos)
    out_leg = None
    if args.output_steps > 0:
        out_leg = output_leg(decs, streams, out_pos, args.output_steps, workers)
        out_leg["vs_headline"] = round(out_leg["fps"] / fps, 3)

    # one stream alone (latency-bound) on the same frames
    sync()
    t1 = time.perf_counter()
    p0 = out_pos[0]
    for t in range(p0, p0 + args.steps):
        lead.decode_prepared(handles[0][t % F])
    lead.synchronize()
    single_fps = args.steps / (time.perf_counter() - t1)

    # host-inclusive rate: batches from host memory (validate + schedule + H2D per frame)
    n_host = min(F, 24)
    t1 = time.perf_counter()
    for i in range(n_host):
        lead.decode_frame(streams[0][i])
    lead.synchronize()
    host_fps = n_host / (time.perf_counter() - t1)
    levels, _ = lead.last_frame_stats()

    # the same with every stream fed by its own host thread (contexts are independent and
    # may be driven concurrently: SURVEY.md §8b threading); frames/s over all streams.  A
    # failure here is reported in the line, never fatal to it
    errs = []

    def feed(d, fr):
        try:
            for i in range(n_host):
                d.decode_frame(fr[i % len(fr)])
            d.synchronize()
        except Exception as e:
            errs.append(str(e))
    host_mt_fps = None
    try:
        th = [threading.Thread(target=feed, args=(d, fr)) for d, fr in zip(decs, streams)]
        t1 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        if not errs:
            host_mt_fps = round(S * n_host / (time.perf_counter() - t1), 3)
    except Exception as e:
        errs.append(str(e))


    # ---- configs[4] end to end from IVF bitstreams (parse on the host inside the timed region)
    ivf = None
    if args.ivf_frames > 0 and args.config == "1080p":
        ivf = ivf_leg(decs, ivf_streams(rank, S, args.ivf_frames), args.ivf_frames)
        if dist:
            ivf["fps_all_ranks"] = round(world * ivf["frames"] / max_over_ranks(ivf["elapsed_s"], dist), 3)

    # a key frame alone on the chip (the deep frames the pipeline launches solo)
    kf = key_frame_ms(lead, handles[0][0])
    for d, hs in zip(decs, handles):
        for hd in hs:
            d.release_prepared(hd)
        d.close()

    # ---- configs[3]: 4K, 4x2 tiles (a bounded extra leg of the default run)
    k4 = None
    if args.config == "1080p" and not args.no_4k:
        k4 = leg_4k(local, rank, world, dist, workers, traffic=args.traffic_4k,
                    ivf_frames=min(args.ivf_frames, 8), prime_steps=args.prime_steps)

    copy_peak = None
    try:
        copy_peak = round(copy_peak_gbps(local), 1)
    except Exception as e:  # reported, never fatal to the line
        errs.append(f"copy peak: {e}")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cfps, cn, cdt = cpu_baseline(streams[0], args.cpu_budget)
        cpu = {"value": round(cfps, 4), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"frames 0..{cn - 1} of synthetic {args.config} stream 0 "
                         f"({cn} frames, {cdt:.1f} s): oracle/av1r_oracle.c, -O2, 1 thread",
               "cpu_model": cpu_model(), "host_cores": os.cpu_count()}
        cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
        kb = None
        if args.config == "1080p":
            try:
                kb = box_k()
            except Exception as e:  # reported, never fatal to the line
                errs.append(f"box k: {e}")
        if kb:
            # k measured here, on this host's CPU (same CPU as the oracle timing above)
            ref_eq = cfps * kb["k"]
            cpu.update({"k": kb["k"], "k_source": "measured in this run on " + cpu_model() + ": " + kb["stream"]
                                                   + "; reference -O1, its decode fps incl. its parse",
                        "k_cpu": cpu_model() + " (this host: the same CPU as the oracle timing)",
                        "reference_measured_here": kb,
                        "reference_equivalent_fps": round(ref_eq, 4),
                        "speedup_end_to_end_vs_reference_equivalent": round(ivf["fps"] / ref_eq, 1) if ivf else None,
                        "speedup_headline_vs_reference_equivalent": round(fps / max(ref_eq, 1e-9), 1),
                        "speedup_headline_note": "parse-excluded GPU rate over a parse-inclusive reference rate"})
            if ivf:
                cpu["speedup_end_to_end_vs_reference_measured_here"] = round(ivf["fps"] / kb["reference_fps"], 1)
        elif os.path.exists(cal):
            # the reference cannot travel; k = reference fps / oracle fps on the
            # same frames, measured in the build container (tools/calibrate_k_1080p.py: the
            # writer's 1080p stream, inter-dominated like this GOP; tools/calibrate_k.py: the
            # conformance streams).  The reference's rate includes its parse, the oracle's not.
            cj = json.load(open(cal))
            kk = cj.get("k_1080p", {}).get("k") if args.config == "1080p" else None
            k = kk if kk else cj["k"]
            ref_eq = cfps * k
            cpu.update({"k": k, "k_source": ("profiles/cpu_calibration.json k_1080p: " + cj["k_1080p"]["stream"]
                                             if kk else "profiles/cpu_calibration.json: " + str(cj["frames"]) +
                                             " conformance frames") + "; reference -O1, its decode fps incl. its parse",
                        "k_cpu": cj["cpu_model"] + " (the build container) -- applied to the oracle timed on "
                                 + cpu_model() + ": cross-CPU unless the two are the same",
                        "reference_equivalent_fps": round(ref_eq, 4),
                        # like with like: the GPU decode from bitstreams (parse included) over the
                        # reference's parse-inclusive rate
                        "speedup_end_to_end_vs_reference_equivalent": round(ivf["fps"] / ref_eq, 1) if ivf else None,
                        # the headline replays parsed batches: parse EXCLUDED on the GPU side
                        "speedup_headline_vs_reference_equivalent": round(fps / max(ref_eq, 1e-9), 1),
                        "speedup_headline_note": "parse-excluded GPU rate over a parse-inclusive reference rate"})
        bg = os.path.join(ROOT, "tests", "golden", "bsw.json")
        if os.path.exists(bg) and args.config == "1080p":
            # the reference decoder itself on a 1080p bitstream (tools/bsw_golden.py, build
            # container, 1 core, -O1): measured, not extrapolated
            g = json.load(open(bg))["1080p_s1"]
            cpu["reference_measured_fps_1080p"] = {"value": g["ref_decode_fps"], "stream": "tools/bsw 1080p_s1 "
                                                   f"({g['frames']} frames, {g['bytes']} B)",
                                                   "where": "build container (profiles/cpu_calibration.json CPU), 1 core"}
            if ivf:
                cpu["speedup_end_to_end_vs_reference_measured"] = round(ivf["fps"] / g["ref_decode_fps"], 1)

    if rank == 0:
        names = ["recon", "lf", "cdef", "lr"]
        line = {
            "metric": "frames/sec 1080p 8-bit 4:2:0 at 1/8 GPU; achieved HBM GB/s vs roofline"
            if args.config == "1080p" else "frames/sec 4K 8-bit 4:2:0 (4x2 tiles)",
            "value": round(fps, 3),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{S} independent synthetic {W}x{H} 8-bit 4:2:0 inter streams per GPU "
                                   f"(BASELINE configs[4] share; each {F} frames: 1 key + {F - 1} inter, cycled, "
                                   f"stream j offset by j*{F}/{S} frames; tiles {tiles[0]}x{tiles[1]}; seeds "
                                   f"{seed:#x}+stream), one frame of every stream per step in shared launches; "
                                   f"host-inclusive: each frame validated, scheduled, packed and uploaded from "
                                   f"host memory inside the timed region (native pipeline kept running across priming, warmup and "
                                   f"the timed window: {workers} packing threads, {depth_eff} frames ahead per stream, packing the "
                                   f"frames after the window while it runs; key frames run alone on their stream, overlapping "
                                   f"the other streams' batches); timed frames: {args.steps * S} of which {r['n_key']} key",
                       "host_threads": workers + 1,
                       "cpus_per_rank": len(bound["cpus"]) if bound else None,
                       "rank0_numa_node": bound["numa_node"] if bound else None,
                       "timed_key_frames": r["n_key"],
                       "streams_per_gpu": S, "frames_per_step": S,
                       "parallelism": f"stream-per-GPU x{world}"},
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "measured_copy_peak": copy_peak,
                         "frac_of_copy_peak": round(achieved / copy_peak, 5) if copy_peak else None,
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "bytes_per_frame": int(sb[dominant]),
                         "ms_per_frame": round(per_frame_ms[dominant], 4)},
            "stage_ms_per_frame": {n: round(v, 4) for n, v in per_frame_ms.items()},
            "recon_kernel_ms_per_frame": {n: round(v, 4) for n, v in r["kernel_ms"].items()},
            "key_frame_alone_ms": kf,
            "stage_algorithmic_GBps": {n: round(r["stage_GBps"][n], 2) for n in names},
            "device_only_fps": round(r["device_fps"], 3),
            "host_profile": r["host_profile"],
            "single_stream_fps": round(single_fps, 3),
            "decode_frame_fps_1thread": round(host_fps, 3),
            "decode_frame_fps_threads": host_mt_fps,
            **({"host_threaded_error": errs[0][:160]} if errs else {}),
            "recon_levels_last_frame": levels,
            "output_inclusive": out_leg,
            "ivf_end_to_end": ivf,
            "config_4k": k4,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
