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

    @property
    def kind(self) -> str:
        return self.meta["kind"]

    def params(self) -> SiftParams:
        return SiftParams(double_image_size=bool(self.meta["double_image_size"]),
                          intervals=int(self.meta["intervals"]),
                          max_octaves=int(self.meta["max_octaves"]))

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
