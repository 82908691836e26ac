"""ctypes binding of the MI355X SIFT C-ABI (include/sift_hip.h).

Python-side mirror of the reference entry point
``detect_keypoints_and_descriptors`` (reference src/sift.hh:65-71,
src/sift.cpp:712-776): same parameter names and defaults, keypoints returned
as a numpy structured array whose dtype is byte-identical to the reference
``struct Keypoint`` (168 B, sift.hh:15-23). Errors raise ``RuntimeError``,
the reference's ``std::runtime_error`` convention.

This module loads ``libsift_hip.so`` from this directory and fails loudly if
it is missing: there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, fields

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SIFT_HIP_LIB") or os.path.join(_HERE, "libsift_hip.so")

KP_DTYPE = np.dtype(
    [
        ("x", "<f8"),
        ("y", "<f8"),
        ("octave", "<i4"),
        ("layer", "<i4"),
        ("size", "<f8"),
        ("pori", "<f8"),
        ("desc", "u1", (128,)),
    ]
)
assert KP_DTYPE.itemsize == 168

EXT_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("z", "<i4"), ("octave", "<i4")])

# sift_match_pair (include/sift_hip.h): KeypointMatch (reference sift.hh:55-63)
# as indices into the two keypoint lists plus the distance
MATCH_DTYPE = np.dtype([("i1", "<u4"), ("i2", "<u4"), ("distance", "<f8")])

# input kinds of sift_hip_submit (include/sift_hip.h)
INPUT_F64_HOST, INPUT_F64_DEVICE, INPUT_U8_HOST, INPUT_U8_DEVICE = 0, 1, 2, 3
MAX_BATCH = 16
MAX_INFLIGHT = 8
PROF_PYRAMID, PROF_EXTREMA, PROF_REFINE, PROF_ORIENT, PROF_DESC, PROF_ROWS = 0, 16, 17, 18, 19, 20

ERRORS = {
    0: "ok",
    -1: "invalid argument",
    -2: "unsupported channel count (1 or 3)",
    -3: "image too small for the octave pyramid",
    -4: "HIP runtime error",
    -5: "out of memory",
    -6: "no such HIP device",
    -7: "parameter outside the supported range",
    -8: "invalid call order (no such job / no previous detect / too many jobs in flight)",
    -9: "RCCL unavailable or a collective failed",
    -10: "another rank of the collective failed",
}

# exported symbols declared in include/sift_hip.h
EXPORTS = (
    "sift_params_default",
    "sift_hip_create",
    "sift_hip_destroy",
    "sift_hip_detect",
    "sift_hip_detect_device",
    "sift_hip_free",
    "sift_hip_strerror",
    "sift_hip_submit",
    "sift_hip_wait",
    "sift_hip_fetch",
    "sift_hip_fetch_device",
    "sift_hip_fetch_device_async",
    "sift_hip_verify_slots",
    "sift_hip_comm_unique_id",
    "sift_hip_comm_init_rank",
    "sift_hip_comm_init_all",
    "sift_hip_comm_destroy",
    "sift_hip_comm_rank",
    "sift_hip_allgather_records",
    "sift_hip_detect_batch",
    "sift_hip_match",
    "sift_hip_match_device",
    "sift_hip_last_counts",
    "sift_hip_copy_level",
    "sift_hip_copy_extrema",
    "sift_hip_copy_records_device",
    "sift_hip_last_timing",
    "sift_hip_stream",
    "sift_hip_set_profiling",
    "sift_hip_blur_profile",
    "sift_hip_profile_table",
    "sift_synth_image",
    "sift_ransac_params_default",
    "sift_hip_ransac_homography",
    "sift_hip_ransac_scores",
    "sift_hip_warp_blend",
)


class CRansacParams(ctypes.Structure):
    """sift_ransac_params (include/sift_hip.h)."""
    _fields_ = [
        ("n_hyp", ctypes.c_int),
        ("refine_iters", ctypes.c_int),
        ("threshold", ctypes.c_double),
        ("seed", ctypes.c_uint64),
    ]


class CParams(ctypes.Structure):
    _fields_ = [
        ("double_image_size", ctypes.c_int),
        ("intervals", ctypes.c_int),
        ("window_size", ctypes.c_int),
        ("max_octaves", ctypes.c_int),
        ("init_sigma", ctypes.c_double),
        ("contrast_threshold", ctypes.c_double),
        ("eigen_ratio", ctypes.c_double),
        ("num_bins", ctypes.c_double),
        ("peak_ratio", ctypes.c_double),
        ("ori_sigma_factor", ctypes.c_double),
        ("desc_scale_factor", ctypes.c_double),
        ("write_keypoints_png", ctypes.c_int),
        ("reserved", ctypes.c_int),
    ]


class CCounts(ctypes.Structure):
    _fields_ = [
        ("extrema", ctypes.c_int64),
        ("refined", ctypes.c_int64),
        ("oriented", ctypes.c_int64),
        ("final_n", ctypes.c_int64),
        ("octaves", ctypes.c_int),
        ("levels_per_octave", ctypes.c_int),
        ("octave0_w", ctypes.c_int),
        ("octave0_h", ctypes.c_int),
    ]


@dataclass
class SiftParams:
    """detect_keypoints_and_descriptors parameters (reference sift.hh:65-71)."""

    double_image_size: bool = True
    init_sigma: float = 1.6
    intervals: int = 3
    window_size: int = 3
    contrast_threshold: float = 0.04
    eigen_ratio: float = 10.0
    num_bins: float = 36
    peak_ratio: float = 0.8
    ori_sigma_factor: float = 1.5
    desc_scale_factor: float = 3.0
    max_octaves: int = 0  # extension: 0 = reference formula

    def to_c(self) -> CParams:
        p = CParams()
        for f in fields(self):
            v = getattr(self, f.name)
            setattr(p, f.name, int(v) if isinstance(v, bool) else v)
        p.write_keypoints_png = 0
        return p


_libs: dict = {}


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libsift_hip.so (raises if it has not been built). Other paths
    (alternative builds for A/B runs) load side by side (RTLD_LOCAL)."""
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} not found: build it with `make -C sift-project_amd` "
            "(no CPU fallback exists on the product path)"
        )
    lib = ctypes.CDLL(path)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    lib.sift_params_default.argtypes = [ctypes.POINTER(CParams)]
    lib.sift_hip_create.argtypes = [i, ctypes.POINTER(vp)]
    lib.sift_hip_destroy.argtypes = [vp]
    det_args = [vp, vp, i, i, i, ctypes.POINTER(CParams), ctypes.POINTER(vp),
                ctypes.POINTER(sz), ctypes.POINTER(vp)]
    lib.sift_hip_detect.argtypes = det_args
    lib.sift_hip_detect_device.argtypes = det_args
    lib.sift_hip_free.argtypes = [vp]
    lib.sift_hip_free.restype = None
    lib.sift_hip_strerror.argtypes = [i]
    lib.sift_hip_strerror.restype = ctypes.c_char_p
    lib.sift_hip_submit.argtypes = [vp, ctypes.POINTER(vp), i, i, i, i, i,
                                    ctypes.POINTER(CParams), i, ctypes.POINTER(i)]
    lib.sift_hip_wait.argtypes = [vp, i, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    lib.sift_hip_fetch.argtypes = [vp, i, vp, vp]
    lib.sift_hip_fetch_device.argtypes = [vp, i, vp, sz]
    if hasattr(lib, "sift_hip_fetch_device_async"):  # (absent from older A/B builds)
        lib.sift_hip_fetch_device_async.argtypes = [vp, i, vp, sz, vp, vp]
        lib.sift_hip_verify_slots.argtypes = [vp, vp, i, sz, i, i, i, i, sz, vp, vp]
    if hasattr(lib, "sift_hip_comm_init_all"):  # (absent from older A/B builds)
        lib.sift_hip_comm_unique_id.argtypes = [vp]
        lib.sift_hip_comm_init_rank.argtypes = [vp, i, i, i, ctypes.POINTER(vp)]
        lib.sift_hip_comm_init_all.argtypes = [i, ctypes.POINTER(i), ctypes.POINTER(vp)]
        lib.sift_hip_comm_destroy.argtypes = [vp]
        lib.sift_hip_comm_rank.argtypes = [vp, ctypes.POINTER(i), ctypes.POINTER(i)]
        lib.sift_hip_allgather_records.argtypes = [vp, vp, vp, vp, i, i, vp, sz, vp, vp,
                                                   ctypes.POINTER(sz), vp]
    lib.sift_hip_detect_batch.argtypes = [vp, ctypes.POINTER(vp), i, i, i, i, i,
                                          ctypes.POINTER(CParams), ctypes.POINTER(vp),
                                          ctypes.POINTER(sz), ctypes.POINTER(vp)]
    match_args = [vp, vp, sz, vp, sz, ctypes.c_double, ctypes.POINTER(vp), ctypes.POINTER(sz)]
    lib.sift_hip_match.argtypes = match_args
    lib.sift_hip_match_device.argtypes = match_args
    lib.sift_hip_last_counts.argtypes = [vp, ctypes.POINTER(CCounts)]
    lib.sift_hip_copy_level.argtypes = [vp, i, i, vp, sz, ctypes.POINTER(i), ctypes.POINTER(i)]
    lib.sift_hip_copy_extrema.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    lib.sift_hip_copy_records_device.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    lib.sift_hip_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i]
    lib.sift_hip_stream.argtypes = [vp]
    lib.sift_hip_stream.restype = vp
    lib.sift_hip_set_profiling.argtypes = [vp, i]
    lib.sift_hip_blur_profile.argtypes = [vp, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.c_double), i]
    lib.sift_hip_profile_table.argtypes = [vp, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int64), i]
    lib.sift_synth_image.argtypes = [i, i, i, ctypes.c_int64, ctypes.c_double,
                                     ctypes.c_uint64, vp]
    lib.sift_ransac_params_default.argtypes = [ctypes.POINTER(CRansacParams)]
    lib.sift_ransac_params_default.restype = None
    lib.sift_hip_ransac_homography.argtypes = [vp, vp, vp, sz, ctypes.POINTER(CRansacParams), vp,
                                               vp, ctypes.POINTER(sz)]
    lib.sift_hip_ransac_scores.argtypes = [vp, vp, vp, sz, ctypes.POINTER(CRansacParams), vp]
    lib.sift_hip_warp_blend.argtypes = [vp, ctypes.POINTER(vp), vp, vp, i, i, vp, i, i, vp]
    _libs[path] = lib
    return lib


SIFT_ERR_ARG = -1  # include/sift_hip.h


def _check(st: int) -> None:
    if st != 0:
        msg = load_library().sift_hip_strerror(st).decode()
        raise RuntimeError(f"sift_hip error {st}: {msg}")


def synth_image(w: int, h: int, channels: int = 1, nblobs: int | None = None,
                smax: float = 6.0, seed: int = 42) -> np.ndarray:
    """Deterministic synthetic image (HWC float64, values 0..255)."""
    lib = load_library()
    if nblobs is None:
        nblobs = max(1, (w * h) // 52)  # 1080p -> ~40k blobs
    out = np.empty((h, w, channels) if channels > 1 else (h, w), dtype=np.float64)
    _check(lib.sift_synth_image(w, h, channels, nblobs, smax, seed, out.ctypes.data))
    return out


def _as_hwc(img: np.ndarray):
    a = np.ascontiguousarray(img, dtype=np.float64)
    if a.ndim == 2:
        return a, a.shape[1], a.shape[0], 1
    if a.ndim == 3:
        return a, a.shape[1], a.shape[0], a.shape[2]
    raise ValueError("image must be (H, W) or (H, W, C)")


class Comm:
    """A rank of the native RCCL record exchange (include/sift_hip.h
    sift_hip_comm_*; what a C++ batch driver uses instead of
    torch.distributed)."""

    def __init__(self, handle: ctypes.c_void_p, lib):
        self.lib, self._c = lib, handle

    @staticmethod
    def init_all(devices) -> list:
        """One communicator per device of this process (ncclCommInitAll)."""
        lib = load_library()
        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        _check(lib.sift_hip_comm_init_all(n, devs, hs))
        return [Comm(ctypes.c_void_p(hs[k]), lib) for k in range(n)]

    def rank(self):
        r, n = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.sift_hip_comm_rank(self._c, ctypes.byref(r), ctypes.byref(n)))
        return r.value, n.value

    def allgather_records(self, d_recs: int, ids, counts, max_local: int, d_out: int,
                          cap_out: int, stream: int = 0):
        """Two-phase all-gather (sift_hip_allgather_records): this rank's
        images ids[j] with counts[j] records image-major at device pointer
        d_recs; returns (total, ids, counts) of every rank's entries (rank-
        major, id -1 = empty); the records land at d_out rank-major."""
        _, nranks = self.rank()
        n_local = len(ids)
        ids_a = np.asarray(ids, dtype=np.int64)
        cnt_a = np.asarray(counts, dtype=np.uint64)
        out_ids = np.empty(nranks * max_local, dtype=np.int64)
        out_cnt = np.empty(nranks * max_local, dtype=np.uint64)
        n_out = ctypes.c_size_t()
        _check(self.lib.sift_hip_allgather_records(
            self._c, ctypes.c_void_p(d_recs or None), ids_a.ctypes.data if n_local else None,
            cnt_a.ctypes.data if n_local else None, n_local, max_local,
            ctypes.c_void_p(d_out or None), cap_out, out_ids.ctypes.data, out_cnt.ctypes.data,
            ctypes.byref(n_out), ctypes.c_void_p(stream or None)))
        return n_out.value, out_ids, out_cnt

    def close(self) -> None:
        if self._c:
            self.lib.sift_hip_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One HIP device context (stream + device arena)."""

    def __init__(self, device: int = 0, lib_path: str | None = None):
        self.lib = load_library(lib_path or LIB_PATH)
        self._ctx = ctypes.c_void_p()
        _check(self.lib.sift_hip_create(device, ctypes.byref(self._ctx)))
        self.device = device
        self._jobs = {}

    def close(self) -> None:
        if self._ctx:
            self.lib.sift_hip_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- jobs (submit / wait / fetch): batches of same-shape images, up to
    # MAX_INFLIGHT in flight; results land directly in numpy storage
    def submit(self, images, kind: int, w: int, h: int, c: int = 1,
               params: SiftParams | None = None, desc_f32: bool = False) -> int:
        """Enqueue one job: `images` is a sequence of host arrays (kind *_HOST)
        or device pointers (kind *_DEVICE) of one shape. Host arrays must stay
        alive until wait(); returns the ticket."""
        n = len(images)
        ptrs = (ctypes.c_void_p * n)()
        host = kind in (INPUT_F64_HOST, INPUT_U8_HOST)
        want = np.float64 if kind == INPUT_F64_HOST else np.uint8
        for b, im in enumerate(images):
            if host:
                # the library copies exactly w*h*c elements of this dtype
                if not isinstance(im, np.ndarray) or im.dtype != want or \
                        not im.flags["C_CONTIGUOUS"] or im.size != w * h * c:
                    raise ValueError(f"image {b}: expected a C-contiguous {np.dtype(want).name} "
                                     f"array of {w}x{h}x{c} elements")
                ptrs[b] = im.ctypes.data
            else:
                if not isinstance(im, int):
                    raise ValueError(f"image {b}: device inputs are integer pointers")
                ptrs[b] = im
        p = (params or SiftParams()).to_c()
        t = ctypes.c_int()
        _check(self.lib.sift_hip_submit(self._ctx, ptrs, n, kind, w, h, c, ctypes.byref(p),
                                        1 if desc_f32 else 0, ctypes.byref(t)))
        self._jobs[t.value] = (n, desc_f32, images)
        return t.value

    def wait(self, ticket: int):
        """Per-image keypoint counts of a submitted job (blocks until done)."""
        n, _, _ = self._jobs[ticket]
        counts = (ctypes.c_size_t * n)()
        total = ctypes.c_size_t()
        _check(self.lib.sift_hip_wait(self._ctx, ticket, counts, ctypes.byref(total)))
        return list(counts)

    def fetch(self, ticket: int):
        """(list of per-image keypoint arrays, list of per-image descriptor
        float arrays or None); releases the job."""
        n, want_f32, _ = self._jobs[ticket]
        counts = self.wait(ticket)
        total = sum(counts)
        kps = np.empty(total, dtype=KP_DTYPE)
        df = np.empty((total, 128), dtype=np.float32) if want_f32 else None
        try:
            _check(self.lib.sift_hip_fetch(self._ctx, ticket,
                                           kps.ctypes.data if total else None,
                                           df.ctypes.data if (want_f32 and total) else None))
        finally:
            del self._jobs[ticket]
        offs = np.cumsum([0] + counts)
        k = [kps[offs[b]:offs[b + 1]] for b in range(n)]
        d = [df[offs[b]:offs[b + 1]] for b in range(n)] if want_f32 else None
        return k, d

    def fetch_device(self, ticket: int, dev_ptr: int, cap: int):
        """Final records of a job written to device memory (image-major, cap
        records available); per-image counts. Releases the job."""
        counts = self.wait(ticket)
        self._release_after(ticket, self.lib.sift_hip_fetch_device(
            self._ctx, ticket, ctypes.c_void_p(dev_ptr), cap))
        return counts

    def fetch_device_async(self, ticket: int, dev_ptr: int, cap: int, stream: int = 0,
                           checksum_ptr: int = 0):
        """fetch_device without a host wait: the gather is enqueued on the
        library's stream and `stream` (hipStream_t handle, e.g. a torch
        stream's cuda_stream) is ordered after it; optionally the records'
        64-bit word sum goes to device memory at checksum_ptr. Releases the
        job; returns per-image counts."""
        counts = self.wait(ticket)
        self._release_after(ticket, self.lib.sift_hip_fetch_device_async(
            self._ctx, ticket, ctypes.c_void_p(dev_ptr), cap, ctypes.c_void_p(stream or None),
            ctypes.c_void_p(checksum_ptr or None)))
        return counts

    def _release_after(self, ticket: int, st: int) -> None:
        """Status of a device fetch: the library keeps the job only when
        the caller's capacity was too small (SIFT_ERR_ARG, the job stays
        fetchable); any other outcome released it, so the ticket goes too."""
        if st != SIFT_ERR_ARG:
            del self._jobs[ticket]
        _check(st)

    def verify_slots(self, slots_ptr: int, n_slots: int, slot_bytes: int, hdr_rows: int,
                     count_word: int, sum_word: int, n_sum_words: int, cap_rows: int,
                     bad_ptr: int, stream: int = 0) -> None:
        """Enqueue the exchange check of n_slots record slots (see
        include/sift_hip.h sift_hip_verify_slots)."""
        _check(self.lib.sift_hip_verify_slots(
            self._ctx, ctypes.c_void_p(slots_ptr), n_slots, slot_bytes, hdr_rows, count_word,
            sum_word, n_sum_words, cap_rows, ctypes.c_void_p(bad_ptr),
            ctypes.c_void_p(stream or None)))

    def detect(self, img: np.ndarray, params: SiftParams | None = None, desc_f32: bool = False):
        """detect_keypoints_and_descriptors on a host image (H,W[,C] float64)."""
        a, w, h, c = _as_hwc(img)
        k, d = self.fetch(self.submit([a], INPUT_F64_HOST, w, h, c, params, desc_f32))
        return k[0], (d[0] if desc_f32 else None)

    def detect_u8(self, img: np.ndarray, params: SiftParams | None = None,
                  desc_f32: bool = False):
        """Same from the 8-bit pixels stb decodes (H,W[,C] uint8)."""
        a = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = a.shape[:2]
        c = 1 if a.ndim == 2 else a.shape[2]
        k, d = self.fetch(self.submit([a], INPUT_U8_HOST, w, h, c, params, desc_f32))
        return k[0], (d[0] if desc_f32 else None)

    def detect_device(self, dev_ptr: int, w: int, h: int, c: int = 1,
                      params: SiftParams | None = None, desc_f32: bool = False):
        """Same, with the image already resident in HBM (device pointer)."""
        k, d = self.fetch(self.submit([int(dev_ptr)], INPUT_F64_DEVICE, w, h, c, params,
                                      desc_f32))
        return k[0], (d[0] if desc_f32 else None)

    def detect_batch(self, images, params: SiftParams | None = None, desc_f32: bool = False,
                     kind: int | None = None, shape=None):
        """One job over several same-shape images (host arrays, or device
        pointers with kind=INPUT_*_DEVICE and shape=(w, h, c)); lists of
        per-image results."""
        if kind is None:
            shaped = [_as_hwc(im) for im in images]
            _, w, h, c = shaped[0]
            for b, (_, wb, hb, cb) in enumerate(shaped):
                if (wb, hb, cb) != (w, h, c):
                    raise ValueError(f"image {b} is {wb}x{hb}x{cb}, image 0 is {w}x{h}x{c}: "
                                     "a job's images share one shape")
            return self.fetch(self.submit([a for a, *_ in shaped], INPUT_F64_HOST, w, h, c,
                                          params, desc_f32))
        w, h, c = shape
        return self.fetch(self.submit([int(x) for x in images], kind, w, h, c, params, desc_f32))

    def _match_result(self, out, n):
        try:
            return np.frombuffer(ctypes.string_at(out.value, n.value * 16), dtype=MATCH_DTYPE) \
                .copy() if n.value else np.zeros(0, dtype=MATCH_DTYPE)
        finally:
            self.lib.sift_hip_free(out)

    def match(self, kps1: np.ndarray, kps2: np.ndarray, ratio_threshold: float = 0.75):
        """match_keypoints (reference sift.cpp:783-815) on the GPU: structured
        array (i1, i2, distance) in increasing i1, indices into kps1 / kps2."""
        a = np.ascontiguousarray(kps1, dtype=KP_DTYPE)
        b = np.ascontiguousarray(kps2, dtype=KP_DTYPE)
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.sift_hip_match(self._ctx, a.ctypes.data if len(a) else None, len(a),
                                       b.ctypes.data if len(b) else None, len(b),
                                       ratio_threshold, ctypes.byref(out), ctypes.byref(n)))
        return self._match_result(out, n)

    def match_device(self, d_kps1: int, n1: int, d_kps2: int, n2: int,
                     ratio_threshold: float = 0.75):
        """Same with both record arrays already in HBM (device pointers)."""
        out, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(self.lib.sift_hip_match_device(self._ctx, ctypes.c_void_p(d_kps1), n1,
                                              ctypes.c_void_p(d_kps2), n2, ratio_threshold,
                                              ctypes.byref(out), ctypes.byref(n)))
        return self._match_result(out, n)

    # ---- stitching consumer (sift_stitch.py drives these) --------------------
    def ransac_params(self, n_hyp=None, threshold=None, refine_iters=None, seed=None):
        p = CRansacParams()
        self.lib.sift_ransac_params_default(ctypes.byref(p))
        for k, v in (("n_hyp", n_hyp), ("threshold", threshold),
                     ("refine_iters", refine_iters), ("seed", seed)):
            if v is not None:
                setattr(p, k, v)
        return p

    def ransac_homography(self, src_xy: np.ndarray, dst_xy: np.ndarray, **kw):
        """(H 3x3 with dst ~ H src, inlier mask, n_inliers) by GPU RANSAC."""
        a = np.ascontiguousarray(src_xy, dtype=np.float64).reshape(-1, 2)
        b = np.ascontiguousarray(dst_xy, dtype=np.float64).reshape(-1, 2)
        if a.shape != b.shape:
            raise ValueError("src/dst point counts differ")
        p = self.ransac_params(**kw)
        H = np.zeros(9, dtype=np.float64)
        mask = np.zeros(len(a), dtype=np.uint8)
        n_in = ctypes.c_size_t()
        _check(self.lib.sift_hip_ransac_homography(self._ctx, a.ctypes.data, b.ctypes.data,
                                                   len(a), ctypes.byref(p), H.ctypes.data,
                                                   mask.ctypes.data, ctypes.byref(n_in)))
        return H.reshape(3, 3), mask.astype(bool), n_in.value

    def ransac_scores(self, src_xy: np.ndarray, dst_xy: np.ndarray, **kw) -> np.ndarray:
        a = np.ascontiguousarray(src_xy, dtype=np.float64).reshape(-1, 2)
        b = np.ascontiguousarray(dst_xy, dtype=np.float64).reshape(-1, 2)
        p = self.ransac_params(**kw)
        out = np.zeros(p.n_hyp, dtype=np.int32)
        _check(self.lib.sift_hip_ransac_scores(self._ctx, a.ctypes.data, b.ctypes.data, len(a),
                                               ctypes.byref(p), out.ctypes.data))
        return out

    def warp_blend(self, images, Hinv, out_w: int, out_h: int) -> np.ndarray:
        """Feather-blended panorama (out_h x out_w x c uint8) of HWC uint8
        images, Hinv[i] = image-from-canvas homography of image i."""
        ims = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        ims = [im[:, :, None] if im.ndim == 2 else im for im in ims]
        c = ims[0].shape[2]
        if any(im.shape[2] != c for im in ims):
            raise ValueError("images differ in channel count")
        ptrs = (ctypes.c_void_p * len(ims))(*[im.ctypes.data for im in ims])
        w = np.array([im.shape[1] for im in ims], dtype=np.int32)
        h = np.array([im.shape[0] for im in ims], dtype=np.int32)
        Hs = np.ascontiguousarray(np.asarray(Hinv, dtype=np.float64).reshape(len(ims), 9))
        out = np.zeros((out_h, out_w, c), dtype=np.uint8)
        _check(self.lib.sift_hip_warp_blend(self._ctx, ptrs, w.ctypes.data, h.ctypes.data, c,
                                            len(ims), Hs.ctypes.data, out_w, out_h,
                                            out.ctypes.data))
        return out

    def counts(self) -> dict:
        c = CCounts()
        _check(self.lib.sift_hip_last_counts(self._ctx, ctypes.byref(c)))
        return {f[0]: getattr(c, f[0]) for f in CCounts._fields_}

    def level(self, octave: int, level: int) -> np.ndarray:
        c = self.counts()
        cap = c["octave0_w"] * c["octave0_h"]
        buf = np.empty(cap, dtype=np.float64)
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.sift_hip_copy_level(self._ctx, octave, level, buf.ctypes.data, cap,
                                            ctypes.byref(w), ctypes.byref(h)))
        return buf[: w.value * h.value].reshape(h.value, w.value).copy()

    def extrema(self) -> np.ndarray:
        n = ctypes.c_size_t()
        _check(self.lib.sift_hip_copy_extrema(self._ctx, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=EXT_DTYPE)
        if n.value:
            _check(self.lib.sift_hip_copy_extrema(self._ctx, out.ctypes.data, n.value,
                                                  ctypes.byref(n)))
        return out

    def copy_records_device(self, dev_ptr: int, cap: int) -> int:
        n = ctypes.c_size_t()
        _check(self.lib.sift_hip_copy_records_device(self._ctx, ctypes.c_void_p(dev_ptr), cap,
                                                     ctypes.byref(n)))
        return n.value

    def n_records(self) -> int:
        n = ctypes.c_size_t()
        _check(self.lib.sift_hip_copy_records_device(self._ctx, None, 0, ctypes.byref(n)))
        return n.value

    def host_timing(self) -> dict:
        """Host-side phase wall times (ms) of the last detect."""
        t = (ctypes.c_double * 6)()
        _check(self.lib.sift_hip_last_timing(self._ctx, t, 6))
        return dict(zip(("enqueue", "wait_device", "download", "finalize", "output", "blocked"),
                        list(t)))

    @property
    def stream(self) -> int:
        return self.lib.sift_hip_stream(self._ctx) or 0

    def set_profiling(self, on: bool) -> None:
        _check(self.lib.sift_hip_set_profiling(self._ctx, 1 if on else 0))

    def profile_table(self, reset: bool = False):
        """Per-row (kernel ms, algorithmic bytes, launches): rows PROF_PYRAMID+o
        = pyramid launches of octave o, PROF_EXTREMA = extrema launches."""
        ms = (ctypes.c_double * PROF_ROWS)()
        b = (ctypes.c_double * PROF_ROWS)()
        n = (ctypes.c_int64 * PROF_ROWS)()
        _check(self.lib.sift_hip_profile_table(self._ctx, ms, b, n, 1 if reset else 0))
        return [(ms[r], b[r], n[r]) for r in range(PROF_ROWS)]

    def blur_profile(self, reset: bool = False):
        ms, n, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _check(self.lib.sift_hip_blur_profile(self._ctx, ctypes.byref(ms), ctypes.byref(n),
                                              ctypes.byref(b), 1 if reset else 0))
        return ms.value, n.value, b.value


def detect_keypoints_and_descriptors(img: np.ndarray, double_image_size: bool = True,
                                     init_sigma: float = 1.6, intervals: int = 3,
                                     window_size: int = 3, contrast_threshold: float = 0.04,
                                     eigen_ratio: float = 10.0, num_bins: float = 36,
                                     peak_ratio: float = 0.8, ori_sigma_factor: float = 1.5,
                                     desc_scale_factor: float = 3.0, device: int = 0):
    """Functional mirror of the reference entry point (sift.hh:65-71)."""
    ctx = _default_context(device)
    p = SiftParams(double_image_size, init_sigma, intervals, window_size, contrast_threshold,
                   eigen_ratio, num_bins, peak_ratio, ori_sigma_factor, desc_scale_factor)
    kps, _ = ctx.detect(img, p)
    return kps


def match_keypoints(keypoints1: np.ndarray, keypoints2: np.ndarray,
                    ratio_threshold: float = 0.75, device: int = 0):
    """Functional mirror of match_keypoints (reference sift.hh:73-75)."""
    return _default_context(device).match(keypoints1, keypoints2, ratio_threshold)


_contexts: dict = {}


def _default_context(device: int) -> Context:
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]
