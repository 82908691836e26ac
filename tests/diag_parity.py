"""Stage-by-stage HIP vs oracle diagnostic (run on the GPU box).

usage: python tests/diag_parity.py [WxH[xC] ...]
Prints, per image: pyramid levels bit-identical, extrema set equality,
counts per stage, and the final-keypoint parity statistics.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle_bind import OracleRun  # noqa: E402
from parity import compare_final, final_ok, sort_extrema  # noqa: E402
from sift_hip import Context, SiftParams, synth_image  # noqa: E402


def run_case(ctx, w, h, c, params=None, seed=42):
    img = synth_image(w, h, c, seed=seed)
    t0 = time.time()
    ref = OracleRun(img, params)
    t1 = time.time()
    gk, gdf = ctx.detect(img, params, desc_f32=True)
    t2 = time.time()
    cnt = ctx.counts()
    lv_bad = []
    for o in range(ref.octaves):
        for l in range(ref.levels):
            a = ctx.level(o, l)
            b = ref.level(o, l)
            if a.shape != b.shape or not np.array_equal(a.view(np.uint64), b.view(np.uint64)):
                nd = -1 if a.shape != b.shape else int(np.count_nonzero(a != b))
                lv_bad.append((o, l, nd))
    ge = sort_extrema(ctx.extrema())
    re_ = sort_extrema(ref.extrema)
    ext_eq = len(ge) == len(re_) and np.array_equal(ge, re_)
    r = compare_final(gk, gdf, ref.final, ref.desc_f32)
    print(f"{w}x{h}x{c} params={params}: oracle {t1 - t0:.2f}s gpu {t2 - t1:.3f}s")
    print(f"   levels_bad={lv_bad[:8]} (n={len(lv_bad)}) extrema gpu={len(ge)} ref={len(re_)} "
          f"equal={ext_eq}")
    print(f"   counts gpu={cnt} ref: refined={len(ref.refined)} oriented={len(ref.oriented)} "
          f"final={len(ref.final)}")
    print(f"   final: {r}  OK={final_ok(r)}")
    return final_ok(r) and not lv_bad and ext_eq


def main(argv):
    ctx = Context(0)
    cases = argv or ["64x48", "320x240", "161x117x3", "755x499x3"]
    ok = True
    for cs in cases:
        parts = [int(v) for v in cs.split("x")]
        w, h = parts[0], parts[1]
        c = parts[2] if len(parts) > 2 else 1
        ok &= run_case(ctx, w, h, c)
    ok &= run_case(ctx, 200, 150, 1, SiftParams(double_image_size=False))
    ok &= run_case(ctx, 300, 200, 1, SiftParams(intervals=2))
    print("ALL_OK" if ok else "SOME_FAILED")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
