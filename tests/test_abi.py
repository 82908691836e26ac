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
    for code in range(0, -10, -1):
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


def test_submit_rejects_host_arrays_that_do_not_match_the_shape():
    """The library copies exactly w*h*c elements of the kind's dtype from
    each host pointer: a smaller array, another dtype or a non-contiguous
    view must be refused before the C call (no host out-of-bounds read)."""
    import numpy as np

    from sift_hip import INPUT_F64_HOST, INPUT_U8_HOST, Context

    ctx = object.__new__(Context)  # validation happens before any library call
    ok = np.zeros((10, 20))
    for imgs, kind in (([np.zeros((10, 10))], INPUT_F64_HOST),
                       ([ok, np.zeros((5, 20))], INPUT_F64_HOST),
                       ([ok.astype(np.float32)], INPUT_F64_HOST),
                       ([ok], INPUT_U8_HOST),
                       ([np.zeros((10, 40))[:, ::2]], INPUT_F64_HOST),
                       ([12345], INPUT_F64_HOST)):
        with pytest.raises(ValueError):
            Context.submit(ctx, imgs, kind, 20, 10, 1)
    with pytest.raises(ValueError, match="share one shape"):
        Context.detect_batch(ctx, [ok, np.zeros((11, 20))])


def test_host_u8_packing_pass():
    """The front end's host pass (csrc/host_pack.cpp, pooled AVX2): an Image
    buffer goes up as bytes only if EVERY value survives the u8 round trip
    bit for bit; one fraction, negative, -0.0, NaN or value > 255 anywhere
    (vector body or scalar tail, any chunk) sends the doubles instead."""
    import numpy as np

    lib = load_library()
    f = lib._ZN8sift_amd12host_pack_u8EPKdmPh  # sift_amd::host_pack_u8 (sift_host.h)
    f.restype = ctypes.c_bool
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    rng = np.random.default_rng(3)
    for n in (7, 4096 + 13, (1 << 17) * 3 + 5):
        img = rng.integers(0, 256, size=n).astype(np.float64)
        out = np.empty(n, np.uint8)
        assert f(img.ctypes.data, n, out.ctypes.data)
        assert np.array_equal(out, img.astype(np.uint8))
        for bad in (0.5, -1.0, -0.0, np.nan, 256.0, 1e12, np.inf):
            for pos in (0, n // 2, n - 1):
                b = img.copy()
                b[pos] = bad
                assert not f(b.ctypes.data, n, out.ctypes.data), (n, bad, pos)


def test_host_pack_pool_generations():
    """the pooled pack pass tags task claims with their
    generation, so back-to-back calls of different task counts (images of
    different sizes above 2^17 elements) never run or count another call's
    tasks. Many alternating calls, every result checked."""
    import numpy as np

    lib = load_library()
    f = lib._ZN8sift_amd12host_pack_u8EPKdmPh
    f.restype = ctypes.c_bool
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    rng = np.random.default_rng(11)
    sizes = [(1 << 17) * k + 3 for k in (2, 9, 3, 17, 5)]
    imgs = {n: rng.integers(0, 256, size=n).astype(np.float64) for n in sizes}
    for it in range(300):
        n = sizes[it % len(sizes)]
        out = np.zeros(n, np.uint8)
        assert f(imgs[n].ctypes.data, n, out.ctypes.data)
        assert np.array_equal(out, imgs[n].astype(np.uint8)), (it, n)


def test_comm_entry_points_reject_bad_args_without_gpu():
    """The native RCCL exchange's argument checks need no device."""
    lib = load_library()
    assert lib.sift_hip_comm_init_all(0, None, None) == -1
    assert lib.sift_hip_comm_destroy(None) == -1
    assert lib.sift_hip_comm_rank(None, None, None) == -1
    n = ctypes.c_size_t()
    assert lib.sift_hip_allgather_records(None, None, None, None, 0, 1, None, 0, None, None,
                                          ctypes.byref(n), None) == -1


def test_python_binding_argument_counts_match_the_header():
    """Every argtypes list set by load_library has as many entries as the
    header's declaration has parameters (a wrong count corrupts the call)."""
    lib = load_library()
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for name in EXPORTS:
        m = re.search(r"\b" + name + r"\s*\(([^)]*)\)", src)
        if not m:
            continue
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        fn = getattr(lib, name)
        if fn.argtypes is not None:
            assert len(fn.argtypes) == len(params), name
