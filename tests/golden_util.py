"""Load the reference-generated golden vectors of tests/golden/*.npz."""
from __future__ import annotations

import glob
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN_DIR = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))

from sift_hip import KP_DTYPE, SiftParams, synth_image  # noqa: E402


class Golden:
    def __init__(self, path: str):
        self.path = path
        z = np.load(path, allow_pickle=False)
        self.meta = json.loads(str(z["meta_json"]))
        self.name = self.meta["name"]
        self.final = np.frombuffer(z["final"].tobytes(), dtype=KP_DTYPE).copy()
        self.desc_f32 = z["desc_f32"].astype(np.float32)
        self.extrema = z["extrema"] if "extrema" in z else None
        self.pyr_sha256 = [str(s) for s in z["pyr_sha256"]] if "pyr_sha256" in z else None
        self.sample_idx = z["sample_idx"] if "sample_idx" in z else None
        self._input_u8 = z["input_u8"] if "input_u8" in z else None

    def _array(self, key):
        z = np.load(self.path, allow_pickle=False)
        return z[key] if key in z.files else None

    def full_desc_u8(self):
        """Big goldens: every final keypoint's u8 descriptor [n, 128]."""
        return self._array("desc_u8_all")

    def full_pori(self):
        """Big goldens: every final keypoint's orientation (f64)."""
        return self._array("pori_all")

    def strat_sample(self):
        """Big goldens: (indices, normalised descriptor floats) of a
        4096-keypoint stratified sample, or (None, None)."""
        return self._array("strat_idx"), self._array("strat_desc_f32")

    @property
    def kind(self) -> str:
        return self.meta["kind"]

    def params(self) -> SiftParams:
        """Every detect argument the reference ran with (sift.hh:65-71)."""
        p = self.meta.get("params")
        if p is None:  # goldens made with the defaults but these three
            return SiftParams(double_image_size=bool(self.meta["double_image_size"]),
                              intervals=int(self.meta["intervals"]),
                              max_octaves=int(self.meta["max_octaves"]))
        return SiftParams(double_image_size=bool(p["double_image_size"]),
                          init_sigma=float(p["init_sigma"]), intervals=int(p["intervals"]),
                          window_size=int(p["window_size"]),
                          contrast_threshold=float(p["contrast_threshold"]),
                          eigen_ratio=float(p["eigen_ratio"]), num_bins=float(p["num_bins"]),
                          peak_ratio=float(p["peak_ratio"]),
                          ori_sigma_factor=float(p["ori_sigma_factor"]),
                          desc_scale_factor=float(p["desc_scale_factor"]),
                          max_octaves=int(p["max_octaves"]))

    def input(self) -> np.ndarray:
        m = self.meta
        if self._input_u8 is not None:
            img = self._input_u8.astype(np.float64)
        else:
            img = synth_image(m["w"], m["h"], m["c"], nblobs=m["nblobs"], smax=m["smax"],
                              seed=m["seed"])
        got = hashlib.sha256(np.ascontiguousarray(img, "<f8").tobytes()).hexdigest()
        assert got == m["input_sha256"], f"{self.name}: input regeneration mismatch"
        return img

    def level_hashes(self):
        """Per-level sha256 list indexed [octave][level]."""
        L = self.meta["levels"]
        return [self.pyr_sha256[o * L:(o + 1) * L] for o in range(self.meta["octaves"])]


def all_goldens(kinds=("small", "medium", "big")):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))):
        if os.path.basename(p) == "match_cases.npz":  # matcher goldens (test_match.py)
            continue
        g = Golden(p)
        if g.kind in kinds:
            out.append(g)
    return out


def sha256_array(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


COORD_FIELDS = ("x", "y", "octave", "layer", "size")


def coords_sha256(kps: np.ndarray) -> str:
    """sha256 over the bit-exact fields of a final keypoint list, in order:
    per keypoint x, y (f8), octave, layer (i4), size (f8), little-endian."""
    dt = np.dtype([("x", "<f8"), ("y", "<f8"), ("octave", "<i4"), ("layer", "<i4"),
                   ("size", "<f8")])
    a = np.zeros(len(kps), dtype=dt)
    for f in COORD_FIELDS:
        a[f] = kps[f]
    return hashlib.sha256(a.tobytes()).hexdigest()
