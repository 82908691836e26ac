"""GPU: the native RCCL record exchange of the C-ABI (include/sift_hip.h
sift_hip_comm_* / sift_hip_allgather_records) — what a C++ batch driver uses
to shard BASELINE config 4 without torch. At world size 1 (one
GPU box) it must return the same bytes as the torch path
(sift_dist.allgather_records over RCCL), and the C++ batch driver
(tools/sift_batch_driver, one host thread per GPU) must deliver exactly the
records a direct detect gives. Multi-rank runs are unmeasured on hardware
(the 8-GPU node is the driver's): the same two phases run over gloo in
tests/test_dist.py.

Reference: detect_keypoints_and_descriptors is a pure function of one image
(src/sift.cpp:712-776).
"""
import json
import os
import socket
import subprocess

import numpy as np
import pytest

from sift_hip import Comm, synth_image

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpu_native_allgather_matches_torch_path_world1(gpu_ctx):
    import torch
    import torch.distributed as dist

    from sift_dist import RECORD_BYTES, allgather_records

    dev = torch.device("cuda", 0)
    imgs = [synth_image(480, 360, 1, seed=700 + i) for i in range(3)]
    kps, _ = gpu_ctx.detect_batch(imgs)
    ids = [5, 9, 2]  # global image indices, any order
    counts = [len(k) for k in kps]
    recs = torch.from_numpy(np.concatenate([k.view(np.uint8) for k in kps]).copy()).to(dev)
    n = sum(counts)
    out = torch.full((n + 7, RECORD_BYTES), 0xEE, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    comm = Comm.init_all([0])[0]
    try:
        assert comm.rank() == (0, 1)
        total, out_ids, out_counts = comm.allgather_records(recs.data_ptr(), ids, counts, 4,
                                                            out.data_ptr(), n + 7)
        assert total == n
        assert list(out_ids) == ids + [-1] and list(out_counts) == counts + [0]
        native = out[:n].cpu().numpy().tobytes()
        assert bool((out[n:] == 0xEE).all())
        # too small a destination: the collective completes, the error says so
        with pytest.raises(RuntimeError, match="invalid argument"):
            comm.allgather_records(recs.data_ptr(), ids, counts, 4, out.data_ptr(), n - 1)
        # an empty rank takes part too
        total0, ids0, _ = comm.allgather_records(0, [], [], 4, 0, 0)
        assert total0 == 0 and list(ids0) == [-1] * 4
    finally:
        comm.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        bufs = [torch.from_numpy(k.view(np.uint8).reshape(-1, RECORD_BYTES).copy()).to(dev)
                for k in kps]
        got = allgather_records(bufs, ids, 4)
        via_torch = b"".join(got[i].cpu().numpy().tobytes() for i in ids)
    finally:
        dist.destroy_process_group()
    assert native == via_torch == b"".join(k.tobytes() for k in kps)


@pytest.mark.parametrize("n_gpus", [1, 2])
def test_gpu_cpp_batch_driver(gpu_ctx, n_gpus):
    """tools/sift_batch_driver: images sharded i % n_gpus, one host thread
    per GPU, records to HBM, native exchange; every image's record count and
    the exchanged bytes' word sum equal a direct detect's. With 2 GPUs (skipped
    on a one-GPU box) the 3 images are uneven over the ranks (2 + 1), so the
    padding to the largest rank and the rank-major compaction run for real."""
    import torch

    if torch.cuda.device_count() < n_gpus:
        pytest.skip(f"needs {n_gpus} GPUs")
    exe = os.path.join(ROOT, "tools", "sift_batch_driver")
    assert os.path.exists(exe), "tools/sift_batch_driver not built (__graft_entry__.build())"
    w, h, n = 640, 480, 3
    r = subprocess.run([exe, str(n), str(w), str(h), str(n_gpus)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    kps = [gpu_ctx.detect(synth_image(w, h, 1, seed=42 + i))[0] for i in range(n)]
    assert res["gpus"] == n_gpus and res["ranks_agree"]
    assert res["counts"] == [len(k) for k in kps]
    words = np.frombuffer(b"".join(k.tobytes() for k in kps), dtype=np.uint64)
    assert res["total"] == sum(len(k) for k in kps)
    assert res["checksum"] == int(words.sum(dtype=np.uint64))
