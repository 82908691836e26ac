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

    No count exchange and no host synchronisation on the data path: every
    rank sends a fixed-capacity slot (`cap_rows` records of 168 B after
    header rows) with ``all_gather_into_tensor`` issued asynchronously on a
    side stream, so the exchange overlaps the following steps' detection.
    A slot collects the records of `steps_per_exchange` consecutive steps
    (one collective per bucket of steps: RCCL's per-call host cost is
    amortised; xGMI moves larger messages at the same per-link rate), and
    slots are double-buffered: a slot is refilled only after the collective
    that last read it has completed. `cap_rows` (per slot, i.e. per bucket of
    steps) must be the same on every rank (see ``agree_capacity``). Every
    rank always takes part in the same collectives (no per-rank fallback that
    could diverge): a slot that overflows is sent truncated with its true
    count, and ``result`` raises for it; ``allgather_records`` is the exact
    two-phase exchange for callers that cannot bound the counts.

    Header words: entry count, record count, (image id, record count) per
    entry (up to max_images per step), then one checksum per step: the
    wrapping 64-bit sum of that step's record words, written by the sender
    (on the device by the library under RCCL, on the host under gloo). Every
    received slot is checked against its checksums once its collective has
    completed (on the device with `verify_ctx`, a sift_hip.Context;
    ``mismatches`` reads the count).

    ``push`` takes host buffers (staged through pinned memory); ``push_device``
    takes a submitted detect job and has the library write its final records
    straight into the device slot (sift_hip_fetch_device_async: gathered on
    the GPU from the records in HBM, ordered before the collective by an
    event), so the payload never crosses PCIe.
    """

    def __init__(self, cap_rows: int, device: torch.device, group=None, max_images: int = 16,
                 verify_ctx=None, steps_per_exchange: int = 1):
        self.group = group
        self.world = dist.get_world_size(group)
        self.cap = int(cap_rows)
        self.device = device
        self.cuda = device.type == "cuda"
        self.max_images = int(max_images)
        self.bucket = max(1, int(steps_per_exchange))
        self.max_entries = self.max_images * self.bucket
        self.sum_word = 2 + 2 * self.max_entries
        self.hdr_words = self.sum_word + self.bucket
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
        self.step = 0        # collectives started
        self.cur = None      # slot being filled
        self._reset_fill()

    def _reset_fill(self):
        self.fill = 0        # records in the current slot (truncated at cap)
        self.total = 0       # records pushed into it (true count)
        self.entries = []    # (image id, count)
        self.n_steps = 0     # steps in the current slot
        self.staged = None   # "host" (push) or "device" (push_device)

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
            want = w[self.sum_word:self.sum_word + self.bucket].sum(dtype="<u8")
            if n > self.cap or int(recs.sum(dtype="<u8")) != int(want):
                self.bad += 1
        self.checked += self.world

    def _open_slot(self) -> int:
        """The slot the next step writes into (claimed at a bucket's first
        step, once the collective that last read it has completed)."""
        if self.cur is None:
            s = self.step & 1
            self._wait_slot(s)
            self.cur = s
            self._reset_fill()
            # (host-staged) unused checksum words of a short bucket read as 0
            self.host[s].view(-1)[self.sum_word * 8:self.hdr_words * 8] = 0
        return self.cur

    def _stage(self, how: str) -> None:
        if self.staged not in (None, how):
            raise ValueError("push and push_device cannot share a bucket of steps")
        self.staged = how

    def _header(self) -> torch.Tensor:
        """The host-built header words (before the per-step checksums)."""
        hdr = torch.zeros(self.sum_word, dtype=torch.int64)
        hdr[0] = len(self.entries)
        hdr[1] = self.total
        for j, (i, c) in enumerate(self.entries):
            hdr[2 + 2 * j] = int(i)
            hdr[3 + 2 * j] = int(c)
        return hdr.view(torch.uint8)

    def _add_entries(self, counts: Sequence[int], image_ids: Sequence[int]) -> None:
        if len(counts) > self.max_images:
            raise ValueError(f"{len(counts)} images per step > max_images={self.max_images}")
        self.entries += [(int(i), int(c)) for c, i in zip(counts, image_ids)]
        self.total += sum(int(c) for c in counts)
        self.n_steps += 1

    def _finish_step(self) -> int:
        """Close the step; start the collective when the bucket is full.
        Returns the slot index (its result is valid once flushed)."""
        s = self.cur
        if self.n_steps == self.bucket:
            self._launch()
        return s

    def _launch(self) -> None:
        """Copy the slot's host-written bytes from pinned staging and start
        the all-gather (async on the side stream for cuda)."""
        s = self.cur
        hdr = self._header()
        h = self.host[s]
        h.view(-1)[: hdr.numel()] = hdr
        # host-staged slots (push) go up whole: header, per-step checksums
        # and records; device-filled ones (push_device) only the header words
        # before the checksums, which the library wrote on the device
        n_host_bytes = (hdr.numel() if self.staged == "device"
                        else (self.hdr_rows + self.fill) * RECORD_BYTES)
        if self.cuda:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self.dev[s].view(-1)[:n_host_bytes].copy_(h.view(-1)[:n_host_bytes],
                                                          non_blocking=True)
                self.work[s] = dist.all_gather_into_tensor(self.gathered[s], self.dev[s],
                                                           group=self.group, async_op=True)
                self.work[s].wait()  # orders the side stream after the collective
                if self.verify_ctx is not None:
                    rows = self.cap + self.hdr_rows
                    self.verify_ctx.verify_slots(
                        self.gathered[s].data_ptr(), self.world, rows * RECORD_BYTES,
                        self.hdr_rows, 1, self.sum_word, self.bucket, self.cap,
                        self.bad.data_ptr(), self.stream.cuda_stream)
                    self.checked += self.world
                ev = torch.cuda.Event()
                ev.record(self.stream)
                self.done[s] = ev
        else:
            self.dev[s].view(-1)[:n_host_bytes] = h.view(-1)[:n_host_bytes]
            self.work[s] = dist.all_gather_into_tensor(self.gathered[s], self.dev[s],
                                                       group=self.group, async_op=True)
            self.done[s] = self.work[s]
        self.step += 1
        self.cur = None

    def push(self, local: Sequence[torch.Tensor], image_ids: Sequence[int]) -> int:
        """Add this step's buffers (uint8 [n_i, 168], host) to the exchange;
        returns the slot index whose `gathered` buffer will hold the result."""
        s = self._open_slot()
        self._stage("host")
        h = self.host[s]
        k = self.n_steps
        self._add_entries([int(t.shape[0]) for t in local], image_ids)
        off0 = self.hdr_rows + self.fill
        off = off0
        for t in local:  # a slot that overflows is truncated and flagged
            n = min(int(t.shape[0]), self.cap + self.hdr_rows - off)
            h[off: off + n] = t[:n]
            off += n
        self.fill = off - self.hdr_rows
        words = h[off0: off].numpy().view("<u8")
        h.view(-1)[(self.sum_word + k) * 8:(self.sum_word + k + 1) * 8] = torch.from_numpy(
            np.array([words.sum(dtype="<u8")], dtype="<u8").view(np.uint8))
        return self._finish_step()

    def push_device(self, sift_ctx, ticket: int, image_ids: Sequence[int]) -> int:
        """Add a submitted detect job's records to the exchange: the library
        writes them into the device slot (no host copy of the payload; only
        the header goes through pinned staging) and their checksum into the
        step's header word."""
        counts = sift_ctx.wait(ticket)
        n_rows = sum(counts)
        s = self._open_slot()
        self._stage("device")
        k = self.n_steps
        base = self.dev[s][self.hdr_rows + self.fill:]
        room = self.cap - self.fill
        chk = self.dev[s].view(-1)[(self.sum_word + k) * 8:(self.sum_word + k + 1) * 8]
        if n_rows <= room:
            # gathered on the library's stream; the side stream waits on it
            # with an event (no host synchronisation)
            sift_ctx.fetch_device_async(ticket, base.data_ptr(), room, self.stream.cuda_stream,
                                        chk.data_ptr())
            self.fill += n_rows
        else:  # overflow: truncated and flagged, as push does
            cur = torch.cuda.current_stream(self.device)
            tmp = torch.empty((n_rows, RECORD_BYTES), dtype=torch.uint8, device=self.device)
            sift_ctx.fetch_device_async(ticket, tmp.data_ptr(), n_rows, cur.cuda_stream)
            base[:room].copy_(tmp[:room])
            w = base[:room].reshape(-1).view(torch.int64)  # torch sums int64 with wrap-around
            chk.view(torch.int64).copy_(w.sum().view(1))
            self.fill = self.cap
        self._add_entries(counts, image_ids)
        return self._finish_step()

    def flush(self) -> None:
        """Start the collective of a partly filled bucket, then wait for
        every exchange in flight."""
        if self.cur is not None and self.n_steps > 0:
            if self.staged == "device":  # checksum words of the missing steps
                self.dev[self.cur].view(-1)[(self.sum_word + self.n_steps) * 8:
                                            self.hdr_words * 8].zero_()
            self._launch()
        for s in (0, 1):
            self._wait_slot(s)

    def mismatches(self) -> int:
        """Received slots whose records did not sum to their senders'
        checksums (one check per rank per completed collective); call flush
        first."""
        if self.cuda:
            torch.cuda.synchronize(self.device)
        return int(self.bad.item())

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
