"""Host-side phase timing of detect_device on the 1080p bench image."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))
from sift_hip import Context, synth_image  # noqa: E402

img = synth_image(1920, 1080, 1, seed=42)
t = torch.from_numpy(img).to("cuda:0")
torch.cuda.synchronize()
ctx = Context(0)
for _ in range(3):
    ctx.detect_device(t.data_ptr(), 1920, 1080, 1)
acc = {}
walls = []
for _ in range(20):
    t0 = time.perf_counter()
    kps, _ = ctx.detect_device(t.data_ptr(), 1920, 1080, 1)
    walls.append((time.perf_counter() - t0) * 1e3)
    for k, v in ctx.host_timing().items():
        acc.setdefault(k, []).append(v)
print("python wall ms: median %.3f min %.3f" % (np.median(walls), np.min(walls)))
for k, v in acc.items():
    print(f"  {k:12s} median {np.median(v):.3f} ms  min {np.min(v):.3f}")
print("keypoints", len(kps))
