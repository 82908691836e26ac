"""Interleaved A/B of pipeline variants in ONE process, robust to the slow
drift between runs seen on the GPU boxes (±10 % run to run).

Each variant is a context created under its own environment knobs (read at
sift_hip_create) and/or an alternative library build (SIFT_HIP_LIB=path, see
`make alt` in sift-project_amd/Makefile). Blocks of pipelined 1080p steps run
round-robin over the variants; per variant we report the mean ms per image
and each round's ratio to variant 0.

usage: python tools/ab_interleaved.py [--rounds 8] [--steps 300] VARIANT...
  VARIANT = "base" or comma-separated VAR=value settings
"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))

import torch  # noqa: E402

from sift_hip import INPUT_F64_DEVICE, Context, SiftParams, synth_image  # noqa: E402


def make_ctx(spec: str) -> Context:
    env = {} if spec == "base" else dict(kv.split("=", 1) for kv in spec.split(","))
    lib = env.pop("SIFT_HIP_LIB", None)
    prof = env.pop("PROFILE", None) == "1"  # per-launch pyramid/extrema events on
    depth = int(env.pop("DEPTH", "0"))  # jobs in flight for this variant (0: --depth)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctx = Context(0, lib_path=lib)
        ctx.set_profiling(prof)
        ctx.ab_depth = depth
        return ctx
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def run(ctx, ptrs, W, H, params, n, depth, batch):
    q = collections.deque()
    kp = 0
    t0 = time.perf_counter()
    for k in range(n):
        while len(q) < depth and k + len(q) < n:
            q.append(ctx.submit(ptrs, INPUT_F64_DEVICE, W, H, 1, params))
        kp += sum(len(x) for x in ctx.fetch(q.popleft())[0])
    return (time.perf_counter() - t0) / (n * batch), kp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    W, H = 1920, 1080
    imgs = [torch.from_numpy(synth_image(W, H, 1, seed=42 + i)).cuda() for i in range(a.batch)]
    ptrs = [t.data_ptr() for t in imgs]
    params = SiftParams()
    ctxs = [make_ctx(v) for v in a.variants]
    kps = []
    for c in ctxs:
        run(c, ptrs, W, H, params, 20, a.depth, a.batch)
        kps.append(run(c, ptrs, W, H, params, 3, 1, a.batch)[1])
    if len(set(kps)) != 1:
        print("keypoint counts differ between variants:", kps)
        return 1
    t = collections.defaultdict(list)
    for r in range(a.rounds):
        order = list(range(len(ctxs)))
        if r % 2:
            order.reverse()
        for i in order:
            t[i].append(run(ctxs[i], ptrs, W, H, params, a.steps, ctxs[i].ab_depth or a.depth,
                            a.batch)[0] * 1e3)
    for i, v in enumerate(a.variants):
        ratios = [x / y for x, y in zip(t[i], t[0])]
        print(f"{v:60s} mean {sum(t[i]) / len(t[i]):.4f} ms/img  min {min(t[i]):.4f}  "
              f"ratio-to-0 mean {sum(ratios) / len(ratios):.4f} "
              f"[{min(ratios):.3f}..{max(ratios):.3f}]", flush=True)
    for c in ctxs:
        c.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
