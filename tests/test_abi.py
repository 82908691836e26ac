"""CPU: the C-ABI library loads and exports every symbol include/*.h declares;
struct layouts match the reference Keypoint; no compute calls need a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from sift_hip import EXPORTS, KP_DTYPE, LIB_PATH, CParams, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sift_hip.h")


def declared_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**([a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_binding_exports():
    assert set(declared_functions(HEADER)) == set(EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = load_library()
    for name in declared_functions(HEADER):
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in declared_functions(HEADER):
        assert re.search(rf"\bT {name}$", out, flags=re.M), name


def test_keypoint_layout_matches_reference():
    # reference sift.hh:15-23 — x@0 y@8 octave@16 layer@20 size@24 pori@32 desc@40
    assert KP_DTYPE.itemsize == 168
    assert [KP_DTYPE.fields[f][1] for f in ("x", "y", "octave", "layer", "size", "pori", "desc")] \
        == [0, 8, 16, 20, 24, 32, 40]
    assert ctypes.sizeof(CParams) == 80


def test_params_default_are_reference_defaults():
    lib = load_library()
    p = CParams()
    lib.sift_params_default(ctypes.byref(p))
    assert (p.double_image_size, p.intervals, p.window_size, p.max_octaves) == (1, 3, 3, 0)
    assert (p.init_sigma, p.contrast_threshold, p.eigen_ratio, p.num_bins, p.peak_ratio,
            p.ori_sigma_factor, p.desc_scale_factor) == (1.6, 0.04, 10.0, 36.0, 0.8, 1.5, 3.0)


def test_strerror_covers_codes():
    lib = load_library()
    for code in range(0, -9, -1):
        assert lib.sift_hip_strerror(code).decode() != "unknown error"


def test_null_args_are_rejected_without_gpu():
    lib = load_library()
    n = ctypes.c_size_t()
    assert lib.sift_hip_detect(None, None, 1, 1, 1, None, None, ctypes.byref(n), None) == -1
    assert lib.sift_hip_destroy(None) == -1
    assert lib.sift_hip_last_counts(None, None) == -1


def test_kernels_are_gfx950_code_objects():
    blob = open(LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"k_blur" in blob and b"k_orient" in blob and b"k_descriptor" in blob
