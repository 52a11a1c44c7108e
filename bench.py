#!/usr/bin/env python3
"""bench.py -- frames/s of the MI355X AV1 reconstruction + in-loop filter backend.

Workload (BASELINE.json configs[2]): a synthetic 1920x1080 8-bit 4:2:0 stream of frame
batches (tools/synth: 1 key frame + 59 inter frames, seed 0x5EED0001 + rank, 8-tap subpel,
compound avg/dist/wedge/diff-weighted, inter-intra, OBMC, local warp, LF + CDEF + LR),
cycled.  One "step" = one frame through recon -> deblock -> CDEF -> loop restoration on
one GPU with its batch already resident in HBM (av1r_prepare); the host-inclusive rate
(validation + scheduling + PCIe upload per frame) is reported beside it.

Multi-GPU (--gpus N, launched by torch.distributed.run): every rank decodes its own
independent stream on its own GPU -- streams shard one per GPU with no data-path
collective; a gloo barrier brackets the timed region and the MAX elapsed
over ranks is used.  value = N * steps / max_elapsed ("weak" scaling).

Also reported: roofline of the dominant stage (algorithmic bytes / device time, vs the
8 TB/s HBM3E peak) and the CPU baseline (the C oracle -- a restatement of the
reference's algorithm -- on a bounded sample of the same stream, 1 core).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (width, height, tiles, seed)
    "1080p": (1920, 1080, (1, 1), 0x5EED0001),
    "4k": (3840, 2160, (4, 2), 0x5EED0002),
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--config", default="1080p", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=60, help="stream length (1 key + inter)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo")

    import pysynth
    from av1dec_amd import Decoder, native

    native.lib()
    W, H, tiles, seed = CONFIGS[args.config]
    frames = pysynth.stream(W, H, args.frames, stream_seed(seed, rank), sb128=True, tiles=tiles)

    dec = Decoder(local, keep_stages=False, timing=False)
    dec.set_discard_output(True)
    handles = [dec.prepare(f) for f in frames]
    order = [i % len(frames) for i in range(args.warmup + args.steps)]

    for i in order[:args.warmup]:
        dec.decode_prepared(handles[i])
    dec.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for i in order[args.warmup:]:
        dec.decode_prepared(handles[i])
    dec.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist)
    fps = aggregate_fps(world, args.steps, elapsed)

    # per-stage device time over the same frames (HIP events on the decoder's stream)
    dec.l.av1r_set_timing(dec.c, 1)
    for i in order[args.warmup:]:
        dec.decode_prepared(handles[i])
    totals, nfr = dec.stage_times()
    dec.l.av1r_set_timing(dec.c, 0)
    names = ["recon", "lf", "cdef", "lr"]
    per_frame_ms = {n: totals[k] / max(nfr, 1) for k, n in enumerate(names)}
    sb = {n: 0.0 for n in names}
    for i in order[args.warmup:]:
        for n, v in stage_bytes(frames[i]).items():
            sb[n] += v / args.steps
    dominant = max(names, key=lambda n: per_frame_ms[n])
    achieved = sb[dominant] / (per_frame_ms[dominant] * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            if tj.get("config") == args.config and dominant in tj.get("stages", {}):
                traffic = tj["stages"][dominant]
        except Exception:
            traffic = None

    # host-inclusive rate: batches from host memory (validate + schedule + H2D per frame)
    n_host = min(len(frames), 24)
    dec.synchronize()
    t1 = time.perf_counter()
    for i in range(n_host):
        dec.decode_frame(frames[i])
    dec.synchronize()
    host_fps = n_host / (time.perf_counter() - t1)
    levels, _ = dec.last_frame_stats()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cfps, cn, cdt = cpu_baseline(frames, args.cpu_budget)
        cpu = {"value": round(cfps, 4), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"frames 0..{cn - 1} of the same synthetic {args.config} stream "
                         f"({cn} frames, {cdt:.1f} s): oracle/av1r_oracle.c, -O2, 1 thread"}
    for hd in handles:
        dec.release_prepared(hd)
    dec.close()

    if rank == 0:
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
            "config": {"workload": f"synthetic {W}x{H} 8-bit 4:2:0 inter stream "
                                   f"({args.frames} frames: 1 key + {args.frames - 1} inter, cycled; "
                                   f"tiles {tiles[0]}x{tiles[1]}; seed {seed:#x}+rank)",
                       "frames_per_rank": args.steps, "parallelism": f"stream-per-GPU x{world}"},
            "roofline": {"bound": "hbm", "kernel": dominant, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": traffic,
                         "bytes_per_launch": int(sb[dominant]),
                         "ms_per_launch": round(per_frame_ms[dominant], 4)},
            "stage_ms_per_frame": {n: round(v, 4) for n, v in per_frame_ms.items()},
            "stage_algorithmic_GBps": {n: round(sb[n] / max(per_frame_ms[n], 1e-9) / 1e6, 2) for n in names},
            "host_inclusive_fps": round(host_fps, 3),
            "recon_levels_last_frame": levels,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
