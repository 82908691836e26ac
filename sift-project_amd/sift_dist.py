"""Multi-GPU batch driver pieces: one image per GPU, RCCL all-gather of the
per-image descriptor buffers.

detect_keypoints_and_descriptors is a pure function of one image
(reference src/sift.cpp:712-776), so a batch shards by image with no
data-path collective: rank r processes images {i : i % world == r}. The only
exchange is the all-gather that gives every rank the keypoint records
(168-byte reference Keypoint layout, descriptor included) of every image.
RCCL has no all-gather-v, so counts are gathered first and the payload is
padded to the largest rank (SURVEY §7 "Hard parts").

Works on any torch.distributed backend: "nccl" (= RCCL over xGMI on ROCm)
with device tensors, "gloo" with CPU tensors (the CPU tests).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch
import torch.distributed as dist

RECORD_BYTES = 168


def shard(n_images: int, rank: int, world: int) -> List[int]:
    """Image indices owned by `rank` (round-robin, config 4: i -> GPU i % 8)."""
    return list(range(rank, n_images, world))


def allgather_records(local: Sequence[torch.Tensor], image_ids: Sequence[int],
                      max_local: int, group=None) -> Dict[int, torch.Tensor]:
    """All-gather per-image record buffers.

    local      uint8 tensors of shape [n_i, 168], one per local image, all on
               the same device (the collective's device)
    image_ids  global image index of each local buffer
    max_local  max images per rank (same on every rank)
    Returns {image_id: uint8 [n, 168]} for every image of every rank.
    """
    world = dist.get_world_size(group)
    dev = local[0].device if len(local) else torch.device("cpu")
    if len(local) != len(image_ids) or len(local) > max_local:
        raise ValueError("inconsistent local buffers")
    meta = torch.full((max_local, 2), -1, dtype=torch.int64, device=dev)
    for j, (t, i) in enumerate(zip(local, image_ids)):
        if t.dtype != torch.uint8 or t.dim() != 2 or t.shape[1] != RECORD_BYTES:
            raise ValueError("records must be uint8 [n, 168]")
        meta[j, 0] = int(i)
        meta[j, 1] = t.shape[0]
    metas = [torch.empty_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    rows = [int(m[:, 1].clamp(min=0).sum()) for m in metas]
    max_rows = max(max(rows), 1)
    payload = torch.zeros((max_rows, RECORD_BYTES), dtype=torch.uint8, device=dev)
    if len(local):
        cat = torch.cat(list(local), dim=0)
        payload[: cat.shape[0]] = cat
    gathered = [torch.empty_like(payload) for _ in range(world)]
    dist.all_gather(gathered, payload, group=group)
    out: Dict[int, torch.Tensor] = {}
    for m, buf in zip(metas, gathered):
        off = 0
        for img_id, n in m.tolist():
            if img_id < 0:
                continue
            out[int(img_id)] = buf[off: off + n]
            off += n
    return out
