"""Parity comparison of a HIP result against the oracle / golden vectors.

Contract (BASELINE north star):
  * pyramid levels, extrema set: bit-identical
  * final keypoint count, and per keypoint x, y, octave, layer, size:
    bit-identical (size is recomputed on the host with glibc pow)
  * pori: |d| <= PORI_TOL (device atan2/exp are ocml, not glibc; glibc itself
    is not correctly rounded in ~0.1% of calls, so the last bits of the
    orientation histogram cannot be reproduced exactly)
  * normalised descriptor floats: |d| <= DESC_F32_TOL (1e-4)
  * u8 descriptors: equal except rare +-1 at floor boundaries
"""
from __future__ import annotations

import numpy as np

PORI_TOL = 1e-9
DESC_F32_TOL = 1e-4
DESC_U8_MAX_DIFF = 1
DESC_U8_MAX_FRAC = 1e-3  # fraction of descriptor bytes allowed to differ by 1


def sort_extrema(e: np.ndarray) -> np.ndarray:
    return np.sort(e, order=("octave", "x", "y", "z"))


def compare_final(gk, gdf, rk, rdf) -> dict:
    """Compare final keypoint arrays (both already sorted like clean_keypoints)."""
    out = {"n_gpu": int(len(gk)), "n_ref": int(len(rk))}
    out["count_equal"] = len(gk) == len(rk)
    if not out["count_equal"]:
        return out
    if len(gk) == 0:
        out.update(coords_equal=True, pori_max=0.0, desc_u8_mismatch=0, desc_u8_maxdiff=0,
                   desc_f32_max=0.0)
        return out
    coords = all(
        np.array_equal(gk[f].view(np.uint64) if gk[f].dtype == np.float64 else gk[f],
                       rk[f].view(np.uint64) if rk[f].dtype == np.float64 else rk[f])
        for f in ("x", "y", "octave", "layer", "size"))
    out["coords_equal"] = bool(coords)
    if not coords:
        bad = np.nonzero((gk["x"] != rk["x"]) | (gk["y"] != rk["y"]) |
                         (gk["size"] != rk["size"]) | (gk["octave"] != rk["octave"]) |
                         (gk["layer"] != rk["layer"]))[0]
        out["coords_first_bad"] = int(bad[0]) if len(bad) else -1
        out["coords_n_bad"] = int(len(bad))
    out["pori_max"] = float(np.max(np.abs(gk["pori"] - rk["pori"])))
    out["pori_bitexact_frac"] = float(np.mean(gk["pori"] == rk["pori"]))
    d = np.abs(gk["desc"].astype(np.int32) - rk["desc"].astype(np.int32))
    out["desc_u8_mismatch"] = int(np.count_nonzero(d))
    out["desc_u8_maxdiff"] = int(d.max())
    out["desc_u8_frac"] = float(np.count_nonzero(d)) / d.size
    if gdf is not None and rdf is not None:
        out["desc_f32_max"] = float(np.max(np.abs(gdf.astype(np.float64) - rdf.astype(np.float64))))
    return out


def final_ok(r: dict) -> bool:
    if not r.get("count_equal"):
        return False
    if r["n_ref"] == 0:
        return True
    return (r["coords_equal"] and r["pori_max"] <= PORI_TOL
            and r["desc_u8_maxdiff"] <= DESC_U8_MAX_DIFF
            and r["desc_u8_frac"] <= DESC_U8_MAX_FRAC
            and r.get("desc_f32_max", 0.0) <= DESC_F32_TOL)
