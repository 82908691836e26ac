"""Kernel-alone times per variant: for each variant (environment knobs read at
sift_hip_create, or SIFT_HIP_LIB=alternative build) a SIFT_SERIAL context
runs n synchronous 1080p detects with dispatch-timestamped events (every
kernel alone on the chip) and a normal context measures the synchronous
latency; prints µs per image per kernel family and the latency.

usage: python tools/kernel_alone.py [--n 50] VARIANT...   (VARIANT: base | VAR=v,VAR=v)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))

import torch  # noqa: E402

from sift_hip import (PROF_DESC, PROF_EXTREMA, PROF_ORIENT, PROF_PYRAMID,  # noqa: E402
                      PROF_REFINE, Context, SiftParams, synth_image)


def make(spec: str, serial: bool) -> Context:
    env = {} if spec == "base" else dict(kv.split("=", 1) for kv in spec.split(","))
    lib = env.pop("SIFT_HIP_LIB", None)
    if serial:
        env["SIFT_SERIAL"] = "1"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Context(0, lib_path=lib)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--big", default="", help="a BASELINE config of bench.py (config3, config5)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    if a.big:
        sys.path.insert(0, ROOT)
        import bench  # noqa: E402  (BIG_CONFIGS)
        spec = bench.BIG_CONFIGS[a.big]
        a.w, a.h = spec["w"], spec["h"]
        host = synth_image(a.w, a.h, 1, nblobs=spec["nblobs"], smax=spec["smax"], seed=42)
        p = SiftParams(**spec["params"])
    else:
        host = synth_image(a.w, a.h, 1, seed=42)
        p = SiftParams()
    img = torch.from_numpy(host).cuda()
    torch.cuda.synchronize()
    for v in a.variants:
        c = make(v, True)
        for _ in range(3):
            c.detect_device(img.data_ptr(), a.w, a.h, 1, p)
        c.profile_table(reset=True)
        c.set_profiling(True)
        for _ in range(a.n):
            c.detect_device(img.data_ptr(), a.w, a.h, 1, p)
        c.set_profiling(False)
        t = c.profile_table(reset=True)
        c.close()
        us = lambda rows: sum(r[0] for r in rows) * 1e3 / a.n  # noqa: E731
        per_oct = [r[0] * 1e3 / a.n for r in t[PROF_PYRAMID:PROF_PYRAMID + 16] if r[2]]
        c = make(v, False)
        for _ in range(5):
            c.detect_device(img.data_ptr(), a.w, a.h, 1, p)
        t0 = time.perf_counter()
        for _ in range(a.n):
            kp, _ = c.detect_device(img.data_ptr(), a.w, a.h, 1, p)
        lat = (time.perf_counter() - t0) / a.n * 1e3
        c.close()
        print(f"{v:50s} pyr {us(t[PROF_PYRAMID:PROF_PYRAMID + 16]):7.1f} ext {us([t[PROF_EXTREMA]]):6.1f} "
              f"ref {us([t[PROF_REFINE]]):6.1f} ori {us([t[PROF_ORIENT]]):6.1f} "
              f"desc {us([t[PROF_DESC]]):6.1f} us/img alone | latency {lat:.3f} ms | kp {len(kp)} | "
              f"per-octave pyr " + " ".join(f"{x:.1f}" for x in per_oct), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
