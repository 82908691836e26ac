#!/usr/bin/env python
"""Timeline of a BASELINE config-3 / config-5 leg (bench.py big_config_leg's
shape) for rocprofv3 and for the host side: every job's submit / fetch /
done time and the library's host phases of each job.

usage: python tools/big_profile.py config5 [--images N] [--depth D] [--sync]
Prints one JSON line (stdout); run under
`rocprofv3 --kernel-trace --stats -- python3 tools/big_profile.py ...`
for the kernel timeline.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from sift_hip import INPUT_F64_DEVICE, Context, SiftParams, synth_image  # noqa: E402


def main() -> int:
    import bench  # noqa: E402  (BIG_CONFIGS)

    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=sorted(bench.BIG_CONFIGS))
    ap.add_argument("--images", type=int, default=12)
    ap.add_argument("--depth", type=int, default=bench.BIG_DEPTH)  # as the bench legs
    ap.add_argument("--warmup", type=int, default=-1,
                    help="warm-up jobs (default depth + 2: every slot the pipeline cycles "
                         "through has run one)")
    ap.add_argument("--sync", action="store_true")
    args = ap.parse_args()
    spec = bench.BIG_CONFIGS[args.config]
    w, h = spec["w"], spec["h"]
    p = SiftParams(**spec["params"])
    img = synth_image(w, h, 1, nblobs=spec["nblobs"], smax=spec["smax"], seed=42)
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(img).to(dev)
    torch.cuda.synchronize()
    ptr = [t.data_ptr()]
    c = Context(0)
    depth = 1 if args.sync else args.depth

    def run(n, log):
        q = collections.deque()
        kp = 0
        t0 = time.perf_counter()
        for k in range(n):
            while len(q) < depth and k + len(q) < n:
                a = time.perf_counter()
                q.append(c.submit(ptr, INPUT_F64_DEVICE, w, h, 1, p))
                if log is not None:
                    log.append({"job": k + len(q) - 1, "submit_ms": (a - t0) * 1e3,
                                "submit_cost_ms": (time.perf_counter() - a) * 1e3})
            a = time.perf_counter()
            kps, _ = c.fetch(q.popleft())
            b = time.perf_counter()
            kp += sum(len(x) for x in kps)
            if log is not None:
                log.append({"job": k, "fetch_ms": (a - t0) * 1e3, "done_ms": (b - t0) * 1e3,
                            "host": c.host_timing()})
        return kp, time.perf_counter() - t0

    run(args.warmup if args.warmup >= 0 else depth + 2, None)
    log = []
    kp, dt = run(args.images, log)
    c.close()
    out = {"config": args.config, "images": args.images, "depth": depth,
           "ms_per_image": dt / args.images * 1e3, "keypoints_per_image": kp // args.images,
           "log": log}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
