"""Multi-process (gloo, world_size 2, CPU) coverage of the N>1 bench path: streams shard
one per rank with no data-path collective; only the timing uses a MAX reduction."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        elapsed = 1.0 + rank  # rank 1 is the slow one
        m = bench.max_over_ranks(elapsed, dist)
        q.put((rank, m, bench.aggregate_fps(world, 60, m), bench.stream_seed(0x5EED0001, rank)))
    finally:
        dist.destroy_process_group()


def test_two_rank_timing_and_sharding():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank sees the max elapsed; value = all ranks' frames / that time
    assert [r[1] for r in res] == [2.0, 2.0]
    assert res[0][2] == pytest.approx(2 * 60 / 2.0)
    # independent streams per rank
    assert res[0][3] != res[1][3]


def test_single_rank_passthrough():
    assert bench.max_over_ranks(1.5, None) == 1.5
    assert bench.aggregate_fps(1, 60, 2.0) == 30.0


def _shard_worker(rank, world, port, q):
    """One rank of the bench's N>1 path on real data: it builds ITS shard with the bench's
    own selection (bench.rank_streams), decodes it with the CPU oracle, and reports the
    per-stream output digests.  The only collective is the test's own check that the shards
    are disjoint (the bench itself exchanges nothing but the timing MAX)."""
    import hashlib
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, os.path.join(bench.ROOT, "oracle"))
        import pyoracle
        import torch
        S = 2
        ids = bench.rank_stream_ids(rank, S)
        shard = bench.rank_streams("1080p", rank, S, 2, width=128, height=96)
        digests = []
        for frames in shard:
            o = pyoracle.Oracle(keep_stages=False)
            h = hashlib.md5()
            for fr in frames:
                o.decode_frame(fr)
                while o.output_pending():
                    for plane in o.get_output():
                        h.update(plane.tobytes())
            o.close()
            digests.append(h.hexdigest())
        gathered = [torch.zeros(S, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(gathered, torch.tensor(ids, dtype=torch.int64))
        q.put((rank, ids, digests, [g.tolist() for g in gathered]))
    finally:
        dist.destroy_process_group()


def test_two_rank_real_shards():
    """world_size 2: rank r decodes streams r*S .. r*S+S-1 (disjoint, covering 0..2S-1) and
    gets exactly what one process decoding those streams gets."""
    import hashlib
    import sys
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    all_ids = [i for _, ids, _, _ in res for i in ids]
    assert sorted(all_ids) == list(range(2 * world)) and len(set(all_ids)) == len(all_ids)
    assert res[0][3] == res[1][3] == [r[1] for r in res]
    # single-process reference of the same global streams
    sys.path.insert(0, os.path.join(bench.ROOT, "oracle"))
    import pyoracle
    W, H, tiles, seed = bench.CONFIGS["1080p"]
    import pysynth
    for rank, ids, digests, _ in res:
        for i, d in zip(ids, digests):
            frames = pysynth.stream(128, 96, 2, bench.stream_seed(seed, i), sb128=True, tiles=tiles)
            o = pyoracle.Oracle(keep_stages=False)
            h = hashlib.md5()
            for fr in frames:
                o.decode_frame(fr)
                while o.output_pending():
                    for plane in o.get_output():
                        h.update(plane.tobytes())
            o.close()
            assert h.hexdigest() == d, f"rank {rank} stream {i}"
    assert len({d for _, _, ds, _ in res for d in ds}) == 2 * world  # the shards differ


def test_bench_gpus_2_launches_two_ranks():
    """`bench.py --gpus 2` from a plain shell (no torch.distributed.run): the script starts two
    rank processes itself, each builds its own disjoint shard with the real run's selection,
    and rank 0's line says n_gpus 2 with every rank's stream ids (--dry-run: no GPU)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--streams", "8"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "stream-per-GPU x2"
    sh = sorted(line["shards"], key=lambda s: s["rank"])
    assert [s["rank"] for s in sh] == [0, 1] and [s["local_rank"] for s in sh] == [0, 1]
    assert sh[0]["pid"] != sh[1]["pid"]  # two processes
    assert sh[0]["stream_ids"] == list(range(8)) and sh[1]["stream_ids"] == list(range(8, 16))
    assert sh[0]["digest"] != sh[1]["digest"]  # different streams
    # each rank's host threads on CPUs of its own (the pipeline's threads inherit them)
    c0, c1 = set(sh[0]["cpus"]), set(sh[1]["cpus"])
    assert c0 and c1 and not c0 & c1
    assert c0 | c1 <= set(os.sched_getaffinity(0))
    assert all(s["host_workers"] == max(1, min(len(s["cpus"]), 32) - 1) for s in sh)


def test_rank_cpu_split_by_numa_node():
    """bench.split_rank_cpus: ranks whose GPUs share a NUMA node divide that node's allowed CPUs;
    a rank alone on its node takes all of them; an unknown node (-1) shares the allowed set."""
    node = {0: list(range(0, 8)), 1: list(range(8, 16))}.get
    allowed = set(range(16))
    nodes = [0, 0, 1, 1, 1, 0]
    sets = [bench.split_rank_cpus(allowed, nodes, r, node) for r in range(6)]
    assert sets[0] == [0, 1] and sets[1] == [2, 3, 4] and sets[5] == [5, 6, 7]
    assert sets[2] == [8, 9] and sets[3] == [10, 11, 12] and sets[4] == [13, 14, 15]
    assert bench.split_rank_cpus(allowed, [1], 0, node) == list(range(8, 16))
    assert bench.split_rank_cpus({0, 1}, [1, 1], 1, node) == [1]  # node not allowed: the allowed set
    assert bench.split_rank_cpus(set(range(4)), [-1, -1], 0, node) == [0, 1]
    assert bench.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]


def test_bench_gpus_mismatch_is_refused():
    """A launcher's WORLD_SIZE must agree with --gpus (the line's n_gpus is the world size)."""
    import subprocess
    import sys
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(bench.ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_all_64_configs4_streams_match_oracle():
    """BASELINE configs[4]: the 64 independent 1080p streams of the 8-GPU job, as the 8 ranks'
    shards (bench.rank_streams(r, 8) for r = 0..7) decoded one shard after another on this
    GPU through the bench's native pipeline (1 key + 3 inter frames of every stream, outputs
    kept); every output frame equals the CPU oracle on the same batches."""
    import hashlib
    import sys
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(bench.ROOT, "oracle"))
    import pyoracle
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import run_native

    def md5s(planes_list):
        return [b"".join(hashlib.md5(p.tobytes()).digest() for p in planes) for planes in planes_list]

    def oracle(frames):
        o = pyoracle.Oracle(keep_stages=False)
        out = []
        try:
            for f in frames:
                o.decode_frame(f)
                while o.output_pending():
                    out.append(o.get_output())
        finally:
            o.close()
        return md5s(out)

    S, F, world = 8, 4, 8
    seen = set()
    with ThreadPoolExecutor(16) as ex:
        for rank in range(world):
            ids = bench.rank_stream_ids(rank, S)
            assert not seen & set(ids)
            seen |= set(ids)
            streams = bench.rank_streams("1080p", rank, S, F)
            ref = [ex.submit(oracle, s) for s in streams]
            decs = [Decoder(0, keep_stages=False) for _ in range(S)]
            try:
                st = run_native(decs, "cycle", streams, [0] * S, max_frames=F)
                assert st["frames"] == S * F
                got = []
                for d in decs:
                    outs = []
                    while d.output_pending():
                        outs.append(d.get_output())
                    got.append(md5s(outs))
            finally:
                for d in decs:
                    d.close()
            for j, r in enumerate(ref):
                assert got[j] == r.result(), f"stream {ids[j]} (rank {rank} shard)"
    assert seen == set(range(64))


GOLDEN_GOP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs4_gop_md5.json")


def test_configs4_gop_golden_covers_every_stream():
    """The whole-GOP fixture (tests/golden/make_configs4_gop.py, CPU oracle) holds the 64
    streams of configs[4], 60 output frames each, and its streams' first frames agree with
    the oracle run here on stream 0 (a spot check of the generator)."""
    import json
    g = json.load(open(GOLDEN_GOP))
    assert g["streams"] == 64 and g["frames"] == 60
    assert sorted(int(k) for k in g["md5"]) == list(range(64))
    assert all(len(v) == 60 and len(set(v)) > 1 for v in g["md5"].values())
    # different seeds, different pictures
    assert len({v[0] for v in g["md5"].values()}) == 64


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_configs4_whole_gop_matches_golden():
    """BASELINE configs[4] over a whole GOP: the 64 streams as the 8 ranks' shards
    (bench.rank_streams(r, 8), 60 frames each: the key frame and all 59 inter frames, so
    every frame's references are the GPU's own earlier outputs), decoded one shard after
    another on this GPU through the bench's native pipeline; every output frame's hash equals
    the CPU oracle's (tests/golden/configs4_gop_md5.json, made by make_configs4_gop.py)."""
    import hashlib
    import json
    from concurrent.futures import ThreadPoolExecutor
    from av1dec_amd import Decoder
    from av1dec_amd.pipeline import run_native

    g = json.load(open(GOLDEN_GOP))["md5"]
    S, F, world = 8, 60, 8

    def h(planes):
        return hashlib.md5(b"".join(hashlib.md5(p.tobytes()).digest() for p in planes)).hexdigest()

    with ThreadPoolExecutor(16) as ex:
        for rank in range(world):
            ids = bench.rank_stream_ids(rank, S)
            streams = bench.rank_streams("1080p", rank, S, F)
            decs = [Decoder(0, keep_stages=False) for _ in range(S)]
            try:
                st = run_native(decs, "cycle", streams, [0] * S, max_frames=F)
                assert st["frames"] == S * F
                for j, d in enumerate(decs):
                    outs = []
                    while d.output_pending():
                        outs.append(d.get_output())
                    got = list(ex.map(h, outs))
                    assert got == g[str(ids[j])], f"stream {ids[j]} (rank {rank} shard)"
            finally:
                for d in decs:
                    d.close()
            print(f"configs[4] GOP: rank {rank} shard ({S} streams x {F} frames) equal", flush=True)
