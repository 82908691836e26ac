"""CPU: the multi-GPU batch path (image sharding + all-gather of descriptor
buffers) with torch.distributed gloo, world_size 2 and 3."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle_bind import OracleRun
from sift_dist import RECORD_BYTES, RecordExchange, agree_capacity, allgather_records, shard
from sift_hip import synth_image


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_images, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard(n_images, rank, world)
        max_local = (n_images + world - 1) // world
        bufs = []
        for i in mine:
            # the CPU oracle stands in for the GPU detect on this CPU test
            img = synth_image(96, 72, 1, seed=1000 + i)
            fin = OracleRun(img).final
            bufs.append(torch.from_numpy(np.frombuffer(fin.tobytes(), np.uint8)
                                         .reshape(-1, RECORD_BYTES).copy()))
        got = allgather_records(bufs, mine, max_local)
        out_q.put((rank, {k: v.numpy().tobytes() for k, v in got.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_images", [(2, 5), (3, 7), (2, 2), (3, 2)])
def test_allgather_records_gloo(world, n_images):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_images, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = {i: OracleRun(synth_image(96, 72, 1, seed=1000 + i)).final.tobytes()
              for i in range(n_images)}
    for r in range(world):
        assert results[r] == expect


def test_shard_is_a_partition():
    for world in (1, 2, 4, 8):
        seen = sorted(i for r in range(world) for i in shard(64, r, world))
        assert seen == list(range(64))
        assert all(len(shard(64, r, world)) == 64 // world for r in range(world))


def _records(step, image, n):
    g = np.random.default_rng(step * 1000 + image)
    return g.integers(0, 256, size=(n, RECORD_BYTES), dtype=np.uint8)


def _exchange_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = shard(2 * world, rank, world)  # two images per rank
        cap = agree_capacity(40 + 10 * rank, torch.device("cpu"), slack=1.0)
        ex = RecordExchange(cap, torch.device("cpu"))
        got = []
        sizes = [(5, 7), (0, 3), (cap // 2, cap // 2 + 1)]  # last step overflows: fallback
        for step, (a, b) in enumerate(sizes):
            bufs = [torch.from_numpy(_records(step, ids[0], a + rank)),
                    torch.from_numpy(_records(step, ids[1], b))]
            s = ex.push(bufs, ids)
            ex.flush()
            try:
                got.append({k: v.numpy().tobytes() for k, v in ex.result(s).items()})
            except RuntimeError:
                got.append(None)
        # per-step checksums: the two overflowing slots of the last step are
        # flagged; then a corrupted record byte in a received slot is caught
        checks = [ex.checked, ex.mismatches()]
        ex.gathered[1][ex.hdr_rows + 1, 17] ^= 1  # step 1's slot, rank 0's records
        ex._verify_host(1)
        checks.append(ex.mismatches())
        out_q.put((rank, cap, got, checks))
    finally:
        dist.destroy_process_group()


def test_record_exchange_gloo():
    """Pipelined fixed-slot exchange (bench N > 1 path): every rank gets every
    image's records; an overflowing slot is flagged on every receiver."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, cap, got, checks = q.get(timeout=120)
        res[r] = (cap, got)
        assert checks == [3 * world, world, world + 1], checks
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0] == 1024  # max(40, 50) rounded up to 1024
    for step, (a, b) in enumerate([(5, 7), (0, 3)]):
        want = {}
        for r in range(world):
            ids = shard(2 * world, r, world)
            want[ids[0]] = _records(step, ids[0], a + r).tobytes()
            want[ids[1]] = _records(step, ids[1], b).tobytes()
        for r in range(world):
            assert res[r][1][step] == want
    assert res[0][1][2] is None and res[1][1][2] is None


def _many_images_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = shard(12 * world, rank, world)  # 12 images per rank and step
        ex = RecordExchange(4096, torch.device("cpu"), max_images=16)
        bufs = [torch.from_numpy(_records(7, i, 3 + i % 5)) for i in ids]
        s = ex.push(bufs, ids)
        ex.flush()
        out_q.put((rank, {k: v.numpy().tobytes() for k, v in ex.result(s).items()}))
    finally:
        dist.destroy_process_group()


def test_record_exchange_many_images_gloo():
    """More images per step than one 168-byte header row holds (the round-1
    exchange capped a step at 9 images)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_many_images_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {i: _records(7, i, 3 + i % 5).tobytes() for i in range(12 * world)}
    for r in range(world):
        assert res[r] == want


def _bucket_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = shard(2 * world, rank, world)
        ex = RecordExchange(3 * 64, torch.device("cpu"), steps_per_exchange=3)
        slots = []
        for step in range(4):  # one full bucket of 3 steps, then one flushed alone
            bufs = [torch.from_numpy(_records(step, i, 5 + step + rank)) for i in ids]
            slots.append(ex.push(bufs, ids))
        ex.flush()
        # the first bucket's slot was overwritten by no later collective
        got = {k: v.numpy().tobytes() for k, v in ex.result(slots[0]).items()}
        last = {k: v.numpy().tobytes() for k, v in ex.result(slots[3]).items()}
        out_q.put((rank, got, last, ex.step, ex.checked, ex.mismatches()))
    finally:
        dist.destroy_process_group()


def test_record_exchange_bucketed_gloo():
    """steps_per_exchange = 3: three steps' records share one collective (the
    last bucket's image ids win in result()); a partial bucket is sent by
    flush; every received slot passes its per-step checksums."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, got, last, n_coll, checked, bad = q.get(timeout=120)
        res[r] = (got, last)
        assert (n_coll, checked, bad) == (2, 2 * world, 0)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        got, last = res[r]
        for rr in range(world):
            for i in shard(2 * world, rr, world):
                assert got[i] == _records(2, i, 5 + 2 + rr).tobytes()
                assert last[i] == _records(3, i, 5 + 3 + rr).tobytes()


def test_native_exchange_protocol_multirank():
    """The protocol sift_hip_allgather_records runs over RCCL
    (csrc/sift_exchange.h) at world sizes 1-4 on host threads with a
    host-memory transport (tools/exchange_selftest.cpp): padding to the
    largest rank, slot offsets and the rank-major compaction with uneven and
    empty ranks, and injected local failures (bad argument, max_local
    mismatch, allocation / staging failure, too-small output) after which
    every rank returns with the agreed status and none is left in a
    collective (a hang exits 3 via the watchdog)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                       "exchange_selftest")
    if not os.path.exists(exe):
        pytest.skip("tools/exchange_selftest not built (run __graft_entry__.build())")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
    assert r.stdout.count("\nok ") + r.stdout.startswith("ok ") >= 10


def test_bench_gpus_n_launches_one_worker_per_gpu():
    """`bench.py --gpus 2` without a launcher starts torch.distributed.run
    with two workers itself (it never measures one GPU under --gpus N); here,
    without GPUs, the workers fail and the exit status says so. A WORLD_SIZE
    that disagrees with --gpus is an error, not a warning."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    # (small and without the extra legs: on a multi-GPU box the workers run)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps",
                        "1", "--warmup", "1", "--no-big", "--no-extra", "--no-cpu-baseline",
                        "--no-matcher", "--no-alone"], capture_output=True, text=True,
                       timeout=300, env=env)
    assert "torch.distributed.run" in r.stderr and "--nproc-per-node=2" in r.stderr
    if not torch.cuda.is_available():
        assert r.returncode != 0 and r.stdout.strip() == ""
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r2 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                        capture_output=True, text=True, timeout=300, env=env2)
    assert r2.returncode == 2 and "WORLD_SIZE=1" in r2.stderr
