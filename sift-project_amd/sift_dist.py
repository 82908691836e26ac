"""Multi-GPU batch driver pieces: images sharded over GPUs, RCCL all-gather of
the per-image descriptor buffers.

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

import math
from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.distributed as dist

RECORD_BYTES = 168


def collective_device(group=None) -> torch.device:
    """The device this group's collectives run on: the current CUDA (HIP)
    device under nccl (RCCL), the CPU under gloo."""
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def shard(n_images: int, rank: int, world: int) -> List[int]:
    """Image indices owned by `rank` (round-robin, config 4: i -> GPU i % 8)."""
    return list(range(rank, n_images, world))


def allgather_records(local: Sequence[torch.Tensor], image_ids: Sequence[int],
                      max_local: int, group=None, device=None) -> Dict[int, torch.Tensor]:
    """All-gather per-image record buffers (exact two-phase exchange).

    local      uint8 tensors of shape [n_i, 168], one per local image
    image_ids  global image index of each local buffer
    max_local  max images per rank (same on every rank)
    device     the collective's device (default: collective_device(group));
               every rank uses it, also a rank without images
    Returns {image_id: uint8 [n, 168]} for every image of every rank.
    """
    world = dist.get_world_size(group)
    dev = device if device is not None else collective_device(group)
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
        cat = torch.cat([t.to(dev) for t in local], dim=0)
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


class RecordExchange:
    """Pipelined all-gather of per-step record buffers for a steady stream of
    batches (the multi-GPU bench path).

    One collective per step, no count exchange and no host synchronisation:
    every rank sends a fixed-capacity slot (`cap_rows` records of 168 B after
    header rows holding the image count, the record count and per-image
    (image id, record count) pairs for up to `max_images` images), with
    ``all_gather_into_tensor`` issued asynchronously on a side stream, so
    step i's exchange overlaps step i+1's detection. Slots are
    double-buffered; a slot is refilled only after the collective that last
    read it has completed. `cap_rows` must be the same on every rank (see
    ``agree_capacity``). Every rank always takes part in the same collective
    (no per-rank fallback that could diverge): a slot that overflows is sent
    truncated with its true count, and ``result`` raises for it;
    ``allgather_records`` is the exact two-phase exchange for callers that
    cannot bound the counts.

    ``push`` takes host buffers (staged through pinned memory); ``push_device``
    takes a submitted detect job and has the library write its final records
    straight into the device slot (sift_hip_fetch_device: gathered on the GPU
    from the records in HBM), so the payload never crosses PCIe.
    """

    def __init__(self, cap_rows: int, device: torch.device, group=None, max_images: int = 16,
                 verify_ctx=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.cap = int(cap_rows)
        self.device = device
        self.cuda = device.type == "cuda"
        self.max_images = int(max_images)
        # header words: image count, record count, (image id, count) per
        # image, then the sender's checksum of its records (the wrapping
        # 64-bit sum of their 8-byte words): every received slot of every
        # step is checked against it (on the device with `verify_ctx`, a
        # sift_hip.Context, under RCCL; on the host under gloo)
        self.sum_word = 2 + 2 * self.max_images
        self.hdr_words = self.sum_word + 1
        self.hdr_rows = math.ceil(self.hdr_words * 8 / RECORD_BYTES)
        self.verify_ctx = verify_ctx
        self.bad = torch.zeros(1, dtype=torch.int64, device=device)
        self.checked = 0
        rows = self.cap + self.hdr_rows
        pin = self.cuda
        self.host = [torch.zeros((rows, RECORD_BYTES), dtype=torch.uint8, pin_memory=pin)
                     for _ in range(2)]
        self.dev = [torch.zeros((rows, RECORD_BYTES), dtype=torch.uint8, device=device)
                    for _ in range(2)]
        self.gathered = [torch.zeros((self.world * rows, RECORD_BYTES), dtype=torch.uint8,
                                     device=device) for _ in range(2)]
        self.stream = torch.cuda.Stream(device) if self.cuda else None
        self.done = [None, None]  # per slot: event (cuda) / work handle (cpu)
        self.work = [None, None]
        self.step = 0

    def _wait_slot(self, s: int) -> None:
        if self.done[s] is not None:
            if self.cuda:
                self.done[s].synchronize()
            else:
                self.work[s].wait()
                self._verify_host(s)
            self.done[s] = None
            self.work[s] = None

    def _verify_host(self, s: int) -> None:
        rows = self.cap + self.hdr_rows
        g = self.gathered[s].view(self.world, rows * RECORD_BYTES).numpy()
        for r in range(self.world):
            w = g[r].view("<u8")
            n = int(w[1])
            recs = w[self.hdr_rows * RECORD_BYTES // 8:][: min(n, self.cap) * RECORD_BYTES // 8]
            if n > self.cap or int(recs.sum(dtype="<u8")) != int(w[self.sum_word]):
                self.bad += 1
        self.checked += self.world

    def _next_slot(self) -> int:
        s = self.step & 1
        self.step += 1
        self._wait_slot(s)
        return s

    def _header(self, counts: Sequence[int], image_ids: Sequence[int]) -> torch.Tensor:
        """The header words before the checksum (host-built)."""
        if len(counts) > self.max_images:
            raise ValueError(f"{len(counts)} images per step > max_images={self.max_images}")
        hdr = torch.zeros(self.sum_word, dtype=torch.int64)
        hdr[0] = len(counts)
        hdr[1] = sum(int(c) for c in counts)
        for j, (c, i) in enumerate(zip(counts, image_ids)):
            hdr[2 + 2 * j] = int(i)
            hdr[3 + 2 * j] = int(c)
        return hdr.view(torch.uint8)

    def _launch(self, s: int, n_host_bytes: int) -> None:
        """Copy the slot's first n_host_bytes from its pinned staging and
        start the all-gather (async on the side stream for cuda)."""
        if self.cuda:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self.dev[s].view(-1)[:n_host_bytes].copy_(self.host[s].view(-1)[:n_host_bytes],
                                                          non_blocking=True)
                self.work[s] = dist.all_gather_into_tensor(self.gathered[s], self.dev[s],
                                                           group=self.group, async_op=True)
                self.work[s].wait()  # orders the side stream after the collective
                if self.verify_ctx is not None:
                    rows = self.cap + self.hdr_rows
                    self.verify_ctx.verify_slots(
                        self.gathered[s].data_ptr(), self.world, rows * RECORD_BYTES,
                        self.hdr_rows, 1, self.sum_word, self.cap, self.bad.data_ptr(),
                        self.stream.cuda_stream)
                    self.checked += self.world
                ev = torch.cuda.Event()
                ev.record(self.stream)
                self.done[s] = ev
        else:
            self.dev[s].view(-1)[:n_host_bytes] = self.host[s].view(-1)[:n_host_bytes]
            self.work[s] = dist.all_gather_into_tensor(self.gathered[s], self.dev[s],
                                                       group=self.group, async_op=True)
            self.done[s] = self.work[s]

    def push(self, local: Sequence[torch.Tensor], image_ids: Sequence[int]) -> int:
        """Start the exchange of this step's buffers (uint8 [n_i, 168], host);
        returns the slot index whose `gathered` buffer will hold the result."""
        s = self._next_slot()
        h = self.host[s]
        hdr = self._header([int(t.shape[0]) for t in local], image_ids)
        h.view(-1)[: hdr.numel()] = hdr
        off = self.hdr_rows
        for t in local:  # a slot that overflows is truncated and flagged
            n = min(int(t.shape[0]), self.cap + self.hdr_rows - off)
            h[off: off + n] = t[:n]
            off += n
        words = h[self.hdr_rows: off].numpy().view("<u8")
        h.view(-1)[self.sum_word * 8:(self.sum_word + 1) * 8] = torch.from_numpy(
            np.array([words.sum(dtype="<u8")], dtype="<u8").view(np.uint8))
        self._launch(s, off * RECORD_BYTES)
        return s

    def push_device(self, sift_ctx, ticket: int, image_ids: Sequence[int]) -> int:
        """Start the exchange of a submitted detect job's records: the
        library writes them into the device slot (no host copy of the
        payload; only the header goes through pinned staging)."""
        counts = sift_ctx.wait(ticket)
        n_rows = sum(counts)
        s = self._next_slot()
        base = self.dev[s][self.hdr_rows:]
        chk = self.dev[s].view(-1)[self.sum_word * 8:(self.sum_word + 1) * 8]
        if n_rows <= self.cap:
            # gathered on the library's stream; the side stream waits on it
            # with an event (no host synchronisation), and the library adds
            # the records' word sum into the slot's checksum word
            sift_ctx.fetch_device_async(ticket, base.data_ptr(), self.cap,
                                        self.stream.cuda_stream, chk.data_ptr())
        else:  # overflow: truncated and flagged, as push does
            cur = torch.cuda.current_stream(self.device)
            tmp = torch.empty((n_rows, RECORD_BYTES), dtype=torch.uint8, device=self.device)
            sift_ctx.fetch_device_async(ticket, tmp.data_ptr(), n_rows, cur.cuda_stream)
            base.copy_(tmp[: self.cap])
            w = base.view(-1).view(torch.int64)  # torch sums int64 with wrap-around
            chk.view(torch.int64).copy_(w.sum().view(1))
        hdr = self._header(counts, image_ids)
        self.host[s].view(-1)[: hdr.numel()] = hdr
        self._launch(s, hdr.numel())
        return s

    def mismatches(self) -> int:
        """Slots (one per rank per completed step) whose records did not sum
        to their sender's checksum; call flush first."""
        if self.cuda:
            torch.cuda.synchronize(self.device)
        return int(self.bad.item())

    def flush(self) -> None:
        """Wait for every exchange in flight."""
        for s in (0, 1):
            self._wait_slot(s)

    def result(self, s: int) -> Dict[int, torch.Tensor]:
        """{image_id: uint8 [n, 168]} of a completed slot (call flush first)."""
        rows = self.cap + self.hdr_rows
        out: Dict[int, torch.Tensor] = {}
        g = self.gathered[s].view(self.world, rows, RECORD_BYTES)
        for r in range(self.world):
            hdr = g[r, : self.hdr_rows].reshape(-1)[: self.hdr_words * 8].cpu().view(torch.int64)
            if int(hdr[1]) > self.cap:
                raise RuntimeError(f"rank {r} sent {int(hdr[1])} records into a slot of "
                                   f"{self.cap}: raise the capacity (agree_capacity slack)")
            off = self.hdr_rows
            for j in range(int(hdr[0])):
                n = int(hdr[3 + 2 * j])
                out[int(hdr[2 + 2 * j])] = g[r, off: off + n]
                off += n
        return out


def agree_capacity(local_max_rows: int, device: torch.device, slack: float = 1.5,
                   group=None) -> int:
    """Common slot capacity for RecordExchange: the largest per-rank record
    count seen (e.g. over warm-up steps) times `slack`, rounded up to 1024."""
    t = torch.tensor([int(local_max_rows)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    need = int(t.item() * slack) + 1
    return (need + 1023) // 1024 * 1024
