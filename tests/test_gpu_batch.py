"""GPU: jobs of several images (one batched launch per kernel), pipelined
submits, the u8 upload path and the world-size-1 record exchange — each
image's result against the oracle (the reference restated, pinned by the
goldens) or the reference-generated 1080p golden.

Reference: detect_keypoints_and_descriptors is a pure function of one image
(src/sift.cpp:712-776), so every image of a job must come out exactly as if
detected alone. Tolerances as tests/parity.py.
"""
import os
import socket
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from golden_util import all_goldens
from oracle_bind import OracleRun
from parity import compare_final, final_ok
from sift_hip import (INPUT_F64_DEVICE, INPUT_F64_HOST, INPUT_U8_DEVICE, INPUT_U8_HOST, MAX_INFLIGHT,
                      Context,
                      SiftParams,
                      synth_image)

pytestmark = pytest.mark.gpu


def _oracle_finals(imgs, params=None):
    # ctypes releases the GIL: the oracle runs of a batch go in parallel
    def one(img):
        r = OracleRun(img, params)
        out = (r.final, r.desc_f32)
        r.close()
        return out

    with ThreadPoolExecutor(max_workers=min(8, len(imgs))) as ex:
        return list(ex.map(one, imgs))


def _assert_same_records(a, b):
    assert a.tobytes() == b.tobytes()


def test_gpu_batch_small_vs_oracle(gpu_ctx):
    imgs = [synth_image(320, 240, 1, seed=42 + i) for i in range(8)]
    kps, dfs = gpu_ctx.detect_batch(imgs, desc_f32=True)
    refs = _oracle_finals(imgs)
    for b, (k, d, (rk, rd)) in enumerate(zip(kps, dfs, refs)):
        r = compare_final(k, d, rk, rd)
        assert final_ok(r), (b, r)
    # a batch is the same as the images one at a time
    for b in (0, 5):
        k1, _ = gpu_ctx.detect(imgs[b])
        _assert_same_records(kps[b], k1)


def test_gpu_batch_rgb_params_vs_oracle(gpu_ctx):
    p = SiftParams(double_image_size=False, intervals=4)
    imgs = [synth_image(203, 151, 3, seed=7 + i) for i in range(3)]
    kps, dfs = gpu_ctx.detect_batch(imgs, p, desc_f32=True)
    for b, (k, d, (rk, rd)) in enumerate(zip(kps, dfs, _oracle_finals(imgs, p))):
        assert final_ok(compare_final(k, d, rk, rd)), b


def test_gpu_batch_identical_images_dedup_per_image(gpu_ctx):
    # unique (sift.hh:25-27) must never merge records of different images
    img = synth_image(200, 150, 1, seed=9)
    kps, _ = gpu_ctx.detect_batch([img, img, img])
    one, _ = gpu_ctx.detect(img)
    for k in kps:
        _assert_same_records(k, one)


def test_gpu_batch8_1080p_vs_golden_and_oracle(gpu_ctx):
    """BASELINE config 4 layout on one GPU: 8 1080p images in one job; seed 42
    against the reference-generated golden, every image against the oracle."""
    g = [x for x in all_goldens(kinds=("medium",)) if x.name == "synth_1920x1080"][0]
    imgs = [g.input()] + [synth_image(1920, 1080, 1, seed=43 + i) for i in range(7)]
    kps, dfs = gpu_ctx.detect_batch(imgs, desc_f32=True)
    r = compare_final(kps[0], dfs[0], g.final, g.desc_f32)
    assert final_ok(r) and len(kps[0]) == g.meta["final"], r
    refs = _oracle_finals(imgs)
    for b, (k, d, (rk, rd)) in enumerate(zip(kps, dfs, refs)):
        r = compare_final(k, d, rk, rd)
        assert final_ok(r), (b, r)


def test_gpu_pipelined_jobs(gpu_ctx):
    """MAX_INFLIGHT jobs in flight; one more submit is refused; out-of-order
    waits."""
    a = [synth_image(640, 480, 1, seed=s) for s in (1, 2)]
    b = [synth_image(320, 240, 3, seed=3)]
    wa, ha = 640, 480
    ta = gpu_ctx.submit(a, INPUT_F64_HOST, wa, ha, 1)
    tb = gpu_ctx.submit(b, INPUT_F64_HOST, 320, 240, 3)
    fill = [gpu_ctx.submit(b, INPUT_F64_HOST, 320, 240, 3) for _ in range(MAX_INFLIGHT - 2)]
    with pytest.raises(RuntimeError, match="in flight"):
        gpu_ctx.submit(b, INPUT_F64_HOST, 320, 240, 3)
    for t in fill:
        gpu_ctx.fetch(t)
    kb, _ = gpu_ctx.fetch(tb)
    ka, _ = gpu_ctx.fetch(ta)
    _assert_same_records(ka[1], gpu_ctx.detect(a[1])[0])
    _assert_same_records(kb[0], gpu_ctx.detect(b[0])[0])
    # a steady stream: submit k+1 before fetching k
    imgs = [synth_image(480, 360, 1, seed=100 + i) for i in range(5)]
    solo = [gpu_ctx.detect(im)[0] for im in imgs]
    t = gpu_ctx.submit([imgs[0]], INPUT_F64_HOST, 480, 360, 1)
    for i in range(1, 6):
        t_next = gpu_ctx.submit([imgs[i]], INPUT_F64_HOST, 480, 360, 1) if i < 5 else None
        k, _ = gpu_ctx.fetch(t)
        _assert_same_records(k[0], solo[i - 1])
        t = t_next


@pytest.mark.parametrize("depth", [3, 4, 8])
def test_gpu_deep_pipeline_vs_oracle(gpu_ctx, depth):
    """`depth` jobs in flight (one stream each beyond two) of
    mixed shapes and channel counts, fetched in order and one out of order:
    every job equals the oracle and its synchronous result."""
    shapes = [(480, 360, 1), (333, 251, 3), (640, 360, 1), (97, 61, 1)]
    jobs = []
    for i in range(2 * depth):
        w, h, c = shapes[i % len(shapes)]
        jobs.append((synth_image(w, h, c, seed=500 + i), w, h, c))
    solo = [gpu_ctx.detect(im)[0] for im, *_ in jobs]
    q = []
    for i, (im, w, h, c) in enumerate(jobs):
        if len(q) == depth:
            j, t = q.pop(0)
            k, _ = gpu_ctx.fetch(t)
            _assert_same_records(k[0], solo[j])
        q.append((i, gpu_ctx.submit([im], INPUT_F64_HOST, w, h, c)))
    for j, t in reversed(q):  # out of order
        k, _ = gpu_ctx.fetch(t)
        _assert_same_records(k[0], solo[j])
    for j in (0, len(jobs) - 1):
        ref = OracleRun(jobs[j][0])
        k, d = gpu_ctx.detect(jobs[j][0], desc_f32=True)
        assert final_ok(compare_final(k, d, ref.final, ref.desc_f32))


def test_gpu_u8_and_device_inputs(gpu_ctx):
    import torch

    img = synth_image(400, 300, 3, seed=21)
    k64, d64 = gpu_ctx.detect(img, desc_f32=True)
    k8, d8 = gpu_ctx.detect_u8(img.astype(np.uint8), desc_f32=True)
    _assert_same_records(k64, k8)
    assert np.array_equal(d64, d8)
    t8 = torch.from_numpy(img.astype(np.uint8)).to("cuda:0")
    t64 = torch.from_numpy(img).to("cuda:0")
    torch.cuda.synchronize()
    kd, _ = gpu_ctx.detect_batch([t8.data_ptr(), t8.data_ptr()], kind=INPUT_U8_DEVICE,
                                 shape=(400, 300, 3))
    _assert_same_records(kd[0], k64)
    _assert_same_records(kd[1], k64)
    kd, _ = gpu_ctx.detect_batch([t64.data_ptr(), t64.data_ptr()], kind=INPUT_F64_DEVICE,
                                 shape=(400, 300, 3))
    _assert_same_records(kd[1], k64)
    # a non-integer image takes the double upload and still matches the oracle
    frac = synth_image(160, 120, 1, seed=5) + 0.25
    k, d = gpu_ctx.detect(frac, desc_f32=True)
    ref = OracleRun(frac)
    assert final_ok(compare_final(k, d, ref.final, ref.desc_f32))


def test_gpu_small_batch_threshold_keeps_every_octave():
    """with SIFT_BATCH_PX_LOG2 small, octaves built only by the
    LDS kernel must still be searched (final batch starts at o_small)."""
    os.environ["SIFT_BATCH_PX_LOG2"] = "10"
    try:
        ctx = Context(0)
    finally:
        del os.environ["SIFT_BATCH_PX_LOG2"]
    try:
        img = synth_image(640, 360, 1, seed=42)
        k, d = ctx.detect(img, desc_f32=True)
        ref = OracleRun(img)
        assert final_ok(compare_final(k, d, ref.final, ref.desc_f32))
    finally:
        ctx.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpu_batch_record_exchange_world1(gpu_ctx):
    """The config-4 data path at world size 1 over RCCL: a batch through HIP,
    its records through allgather_records and the pipelined RecordExchange."""
    import torch
    import torch.distributed as dist

    from sift_dist import RECORD_BYTES, RecordExchange, allgather_records

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        dev = torch.device("cuda", 0)
        imgs = [synth_image(480, 360, 1, seed=300 + i) for i in range(4)]
        kps, _ = gpu_ctx.detect_batch(imgs)
        ids = list(range(4))
        bufs = [torch.from_numpy(k.view(np.uint8).reshape(-1, RECORD_BYTES).copy()) for k in kps]
        got = allgather_records([b.to(dev) for b in bufs], ids, 4)
        for i in ids:
            assert got[i].cpu().numpy().tobytes() == kps[i].tobytes()
        ex = RecordExchange(4096, dev, verify_ctx=gpu_ctx)
        s = ex.push(bufs, ids)
        ex.flush()
        res = ex.result(s)
        for i in ids:
            assert res[i].cpu().numpy().tobytes() == kps[i].tobytes()
        # device path: the library writes the job's final records straight
        # into the exchange slot (sift_hip_fetch_device), same bytes
        from sift_hip import INPUT_F64_HOST
        for step in range(3):  # both slots, then reuse
            t = gpu_ctx.submit(imgs, INPUT_F64_HOST, 480, 360, 1)
            s = ex.push_device(gpu_ctx, t, ids)
            ex.flush()
            res = ex.result(s)
            for i in ids:
                assert res[i].cpu().numpy().tobytes() == kps[i].tobytes(), (step, i)
        # every received slot of every step matched its sender's checksum
        assert ex.checked == 4 and ex.mismatches() == 0
        # two steps per collective: both steps' records in one slot
        exb = RecordExchange(8192, dev, verify_ctx=gpu_ctx, steps_per_exchange=2)
        for step in range(3):  # one full bucket, then a partial one sent by flush
            t = gpu_ctx.submit(imgs, INPUT_F64_HOST, 480, 360, 1)
            s = exb.push_device(gpu_ctx, t, [10 * step + i for i in ids])
        exb.flush()
        first, last = exb.result(0), exb.result(s)
        for step, res in ((0, first), (1, first), (2, last)):
            for i in ids:
                assert res[10 * step + i].cpu().numpy().tobytes() == kps[i].tobytes(), (step, i)
        assert exb.step == 2 and exb.checked == 2 and exb.mismatches() == 0
        # a flipped record byte is caught, and the check's scratch (left
        # zeroed by every call) gives the restored slot a clean result again
        g = exb.gathered[0]
        rows = exb.cap + exb.hdr_rows
        bad = torch.zeros(1, dtype=torch.int64, device=dev)
        args = (g.data_ptr(), 1, rows * RECORD_BYTES, exb.hdr_rows, 1, exb.sum_word,
                exb.bucket, exb.cap, bad.data_ptr())
        for flip, want in ((False, 0), (True, 1), (True, 1), (False, 1)):
            if flip:
                g[exb.hdr_rows, 5] ^= 1
            torch.cuda.synchronize()
            gpu_ctx.verify_slots(*args)
            torch.cuda.synchronize()
            assert int(bad.item()) == want, (flip, want)
        # too small a destination keeps the job; then it can still be fetched
        t = gpu_ctx.submit(imgs[:1], INPUT_F64_HOST, 480, 360, 1)
        small = torch.empty((1, RECORD_BYTES), dtype=torch.uint8, device=dev)
        with pytest.raises(RuntimeError, match="invalid argument"):
            gpu_ctx.fetch_device(t, small.data_ptr(), 1)
        k, _ = gpu_ctx.fetch(t)
        assert k[0].tobytes() == kps[0].tobytes()
    finally:
        dist.destroy_process_group()


def test_gpu_fetch_device_bulk_and_exported_paths():
    """sift_hip_fetch_device's two index paths. The first job of a
    fresh context has export buffers for 8192 records per lane, so a dense
    image (> 16k records) falls back to one bulk download; the next job runs
    on the grown export buffers. Both device fetches (sync and async with a
    checksum), on two-image jobs with both keypoint lanes, give the bytes of
    the host fetch."""
    import torch

    from sift_hip import INPUT_F64_HOST

    dev = torch.device("cuda", 0)
    imgs = [synth_image(1600, 1200, 1, nblobs=200000, smax=2.0, seed=91 + i) for i in range(2)]
    host = Context(0)
    try:
        ref, _ = host.detect_batch(imgs)
    finally:
        host.close()
    want = b"".join(k.tobytes() for k in ref)
    n = sum(len(k) for k in ref)
    assert len(ref[0]) > 2 * 8192  # more than the fresh export buffers hold
    ctx = Context(0)
    try:
        for job in range(3):  # bulk (fresh buffers), then exported, then async
            t = ctx.submit(imgs, INPUT_F64_HOST, 1600, 1200, 1)
            out = torch.full((n + 5, 168), 0xAB, dtype=torch.uint8, device=dev)
            if job < 2:
                counts = ctx.fetch_device(t, out.data_ptr(), n + 5)
            else:
                chk = torch.zeros(1, dtype=torch.int64, device=dev)
                counts = ctx.fetch_device_async(t, out.data_ptr(), n + 5,
                                                torch.cuda.current_stream().cuda_stream,
                                                chk.data_ptr())
            torch.cuda.synchronize()
            assert counts == [len(k) for k in ref]
            assert out[:n].cpu().numpy().tobytes() == want, job
            assert bool((out[n:] == 0xAB).all())  # nothing written past the records
            if job == 2:
                assert int(chk.item()) == int(out[:n].view(-1).view(torch.int64).sum().item())
    finally:
        ctx.close()


def test_gpu_async_fetch_then_failed_submit_on_same_slot(gpu_ctx):
    """a submit that fails (bad parameters) on a slot whose async
    device gather is still pending must leave the pending flag for the next
    submit, whose streams then wait for the gather before overwriting the
    slot's records. With MAX_INFLIGHT - 1 jobs in flight the freed slot is
    the only free one, so both submits land on it."""
    import torch

    dev = torch.device("cuda", 0)
    w, h = 640, 480
    img = synth_image(w, h, 1, seed=314)
    other = synth_image(w, h, 1, seed=315)
    ref, _ = gpu_ctx.detect(img)
    ref_other, _ = gpu_ctx.detect(other)
    n = len(ref)
    tickets = [gpu_ctx.submit([img], INPUT_F64_HOST, w, h, 1) for _ in range(MAX_INFLIGHT)]
    out = torch.full((n + 3, 168), 0xCD, dtype=torch.uint8, device=dev)
    gpu_ctx.fetch_device_async(tickets[0], out.data_ptr(), n + 3,
                               torch.cuda.current_stream().cuda_stream)
    with pytest.raises(RuntimeError, match="parameter"):
        gpu_ctx.submit([img], INPUT_F64_HOST, w, h, 1, SiftParams(intervals=0))
    t_new = gpu_ctx.submit([other], INPUT_F64_HOST, w, h, 1)
    torch.cuda.synchronize()
    assert out[:n].cpu().numpy().tobytes() == ref.tobytes()
    assert bool((out[n:] == 0xCD).all())
    _assert_same_records(gpu_ctx.fetch(t_new)[0][0], ref_other)
    for t in tickets[1:]:
        _assert_same_records(gpu_ctx.fetch(t)[0][0], ref)
