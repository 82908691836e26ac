"""GPU: the HIP path through the C-ABI against the reference goldens and the
oracle, stage by stage, plus edge cases and full-size properties.

Tolerances (tests/parity.py): pyramid levels, extrema set, final count and
x/y/octave/layer/size bit-exact; pori <= 1e-9; normalised descriptor floats
<= 1e-4; u8 descriptors +-1 on at most 0.1% of bytes.
"""
import zlib

import numpy as np
import pytest

from golden_util import all_goldens, coords_sha256, sha256_array
from oracle_bind import OracleRun
from parity import compare_final, final_ok, sort_extrema

# the f64 descriptor against the reference's floats (both rounded to f32 for
# the goldens): a few f32 ulps of values <= 0.2 + renormalisation
DESC_F64_F32_TOL = 2.5e-7
from sift_hip import EXT_DTYPE, SiftParams, synth_image

pytestmark = pytest.mark.gpu

GOLDENS = all_goldens(kinds=("small", "medium"))
BIG = all_goldens(kinds=("big",))


def _golden_extrema(g):
    ge = np.zeros(len(g.extrema), dtype=EXT_DTYPE)
    for i, f in enumerate(("x", "y", "z", "octave")):
        ge[f] = g.extrema[:, i]
    return sort_extrema(ge)


@pytest.mark.parametrize("g", GOLDENS, ids=[g.name for g in GOLDENS])
def test_gpu_matches_reference_golden(gpu_ctx, g):
    img = g.input()
    kps, df = gpu_ctx.detect(img, g.params(), desc_f32=True)
    c = gpu_ctx.counts()
    m = g.meta
    assert (c["octaves"], c["extrema"], c["refined"], c["oriented"], c["final_n"]) == \
        (m["octaves"], m["extrema"], m["refined"], m["oriented"], m["final"])
    assert np.array_equal(sort_extrema(gpu_ctx.extrema()), _golden_extrema(g))
    r = compare_final(kps, df, g.final, g.desc_f32)
    assert final_ok(r), r
    if g.pyr_sha256 is not None:
        hashes = g.level_hashes()
        for o in range(m["octaves"]):
            for lv in range(m["levels"]):
                assert sha256_array(gpu_ctx.level(o, lv)) == hashes[o][lv], (o, lv)


def check_big_golden(ctx, g):
    """Counts, the whole extrema set (hash), the bit-exact fields of every
    final keypoint (hash), then EVERY keypoint's pori and u8 descriptor
    against the reference's, and the normalised descriptor floats of the
    64-keypoint and 4096-keypoint stratified samples (src/sift.cpp:541-682)."""
    img = g.input()
    kps, df = ctx.detect(img, g.params(), desc_f32=True)
    c = ctx.counts()
    m = g.meta
    assert (c["octaves"], c["extrema"], c["refined"], c["oriented"], c["final_n"]) == \
        (m["octaves"], m["extrema"], m["refined"], m["oriented"], m["final"])
    assert sha256_array(sort_extrema(ctx.extrema()).view("<i4")) == m["extrema_sha256"]
    assert coords_sha256(kps) == m["coords_sha256"]
    sub = kps[g.sample_idx]
    r = compare_final(sub, df[g.sample_idx], g.final, g.desc_f32)
    assert final_ok(r), r
    # every record: the golden's full descriptor / orientation arrays stand
    # in for the reference records whose bit-exact fields the hash pinned
    ref = kps.copy()
    ref["pori"] = g.full_pori()
    ref["desc"] = g.full_desc_u8()
    sidx, sdf = g.strat_sample()
    r = compare_final(kps, None, ref, None)
    r["desc_f32_max"] = float(np.max(np.abs(df[sidx].astype(np.float64) - sdf)))
    assert final_ok(r), r
    # the size the DEVICE computed (it sets the orientation and descriptor
    # windows) equals the reference's glibc size for every keypoint: the
    # kernels' own records, before the host's finalisation, matched to the
    # final ones by (x, y, octave, layer, pori)
    import torch

    n = ctx.n_records()
    buf = torch.empty((n, 168), dtype=torch.uint8, device="cuda:0")
    assert ctx.copy_records_device(buf.data_ptr(), n) == n
    dev = np.frombuffer(buf.cpu().numpy().tobytes(), dtype=kps.dtype)
    key = lambda a: np.stack([a["x"].view(np.uint64), a["y"].view(np.uint64),  # noqa: E731
                              a["octave"].astype(np.uint64), a["layer"].astype(np.uint64),
                              a["pori"].view(np.uint64)], axis=1)
    kd, kf = key(dev), key(kps)
    order = np.lexsort(kd.T[::-1])
    pos = np.searchsorted(np.ascontiguousarray(kd[order]).view([("", np.uint64)] * 5).ravel(),
                          np.ascontiguousarray(kf).view([("", np.uint64)] * 5).ravel())
    match = order[np.minimum(pos, n - 1)]
    assert np.array_equal(kd[match], kf)
    assert np.array_equal(dev["size"][match].view(np.uint64), kps["size"].view(np.uint64))
    return r


@pytest.mark.parametrize("g", BIG, ids=[g.name for g in BIG])
def test_gpu_matches_big_golden(gpu_ctx, g):
    """BASELINE configs 3 (4096^2, 5 octaves x 5 scales) and 5 (8K dense),
    default descriptor (f64 sample math, k_descriptor_split): every u8
    descriptor byte of every keypoint as the reference's but for floor
    boundaries (at most 1e-6 of the bytes, +-1), and the stratified float
    sample to within f32 rounding."""
    r = check_big_golden(gpu_ctx, g)
    print(g.name, r)
    assert r["desc_u8_frac"] <= 1e-6 and r["desc_f32_max"] <= DESC_F64_F32_TOL, r


CASES = [
    ("ragged_67x43", 67, 43, 1, SiftParams()),
    ("rgb_203x151", 203, 151, 3, SiftParams()),
    ("nodbl_rgb_250x190", 250, 190, 3, SiftParams(double_image_size=False)),
    ("int4_180x140", 180, 140, 1, SiftParams(intervals=4)),
    ("int1_150x110", 150, 110, 1, SiftParams(intervals=1)),
    ("win5_170x130", 170, 130, 1, SiftParams(window_size=5)),
    ("bins72_160x120", 160, 120, 1, SiftParams(num_bins=72, peak_ratio=0.5)),
    ("lowthr_160x120", 160, 120, 1, SiftParams(contrast_threshold=0.02, eigen_ratio=5.0)),
    ("oridesc_160x120", 160, 120, 1, SiftParams(ori_sigma_factor=2.0, desc_scale_factor=4.0)),
    ("sigma2_140x100", 140, 100, 1, SiftParams(init_sigma=2.0)),
    ("wide_sigma_90x70", 90, 70, 1, SiftParams(init_sigma=6.5)),  # R > 24: generic blur path
    ("maxoct3_300x220", 300, 220, 1, SiftParams(max_octaves=3)),
    ("tall_33x400", 33, 400, 1, SiftParams()),
    ("wide_600x20", 600, 20, 1, SiftParams()),
]


# Each of these is also pinned to the reference itself: tests/golden/
# case_<name>.npz (every level hash, extrema, final list; generated by the
# reference with all sift.hh:65-71 arguments) runs in
# test_gpu_matches_reference_golden. Here the oracle adds the stage-by-stage
# view (refined / oriented counts, every level compared as a plane).
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_gpu_matches_oracle_stagewise(gpu_ctx, case):
    name, w, h, c, p = case
    img = synth_image(w, h, c, seed=zlib.crc32(name.encode()) & 0xFFFF)
    ref = OracleRun(img, p)
    kps, df = gpu_ctx.detect(img, p, desc_f32=True)
    cnt = gpu_ctx.counts()
    for o in range(ref.octaves):
        for lv in range(ref.levels):
            a, b = gpu_ctx.level(o, lv), ref.level(o, lv)
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (o, lv)
    assert np.array_equal(sort_extrema(gpu_ctx.extrema()), sort_extrema(ref.extrema))
    assert cnt["refined"] == len(ref.refined)
    assert cnt["oriented"] == len(ref.oriented)
    r = compare_final(kps, df, ref.final, ref.desc_f32)
    assert final_ok(r), r


def test_gpu_flat_and_tiny_images(gpu_ctx):
    kps, _ = gpu_ctx.detect(np.full((64, 80), 77.0))
    assert len(kps) == 0 and gpu_ctx.counts()["extrema"] == 0
    kps, _ = gpu_ctx.detect(synth_image(5, 4, 1, nblobs=2, smax=1.0, seed=2))
    assert gpu_ctx.counts()["octaves"] == 1


def test_gpu_error_paths(gpu_ctx):
    with pytest.raises(RuntimeError, match="too small"):
        gpu_ctx.detect(np.zeros((1, 1)))
    with pytest.raises(RuntimeError, match="channel"):
        gpu_ctx.detect(np.zeros((16, 16, 2)))
    with pytest.raises(RuntimeError, match="parameter"):
        gpu_ctx.detect(np.zeros((32, 32)), SiftParams(intervals=0))
    with pytest.raises(RuntimeError, match="parameter"):
        gpu_ctx.detect(np.zeros((32, 32)), SiftParams(window_size=1))
    # non-finite host doubles: rejected (the extrema scan has no NaN
    # semantics; include/sift_hip.h input kinds)
    for bad in (np.nan, np.inf, -np.inf):
        img = synth_image(64, 48, 1, seed=42)
        img[10, 20] = bad
        with pytest.raises(RuntimeError, match="invalid argument"):
            gpu_ctx.detect(img)
    # the context stays usable after errors
    kps, _ = gpu_ctx.detect(synth_image(64, 48, 1, seed=42))
    assert len(kps) > 0


def test_gpu_deterministic_and_device_input(gpu_ctx):
    import torch

    img = synth_image(640, 480, 1, seed=123)
    a, da = gpu_ctx.detect(img, desc_f32=True)
    b, db = gpu_ctx.detect(img, desc_f32=True)
    assert a.tobytes() == b.tobytes() and np.array_equal(da, db)
    t = torch.from_numpy(img).to("cuda:0")
    torch.cuda.synchronize()
    c, dc = gpu_ctx.detect_device(t.data_ptr(), 640, 480, 1, desc_f32=True)
    assert a.tobytes() == c.tobytes() and np.array_equal(da, dc)


def test_gpu_capacity_regrowth(gpu_ctx):
    # a dense small image after a large one exercises arena reuse; a dense
    # large one exercises overflow re-runs of the compaction buffers
    img = synth_image(1024, 768, 1, nblobs=60000, smax=2.0, seed=77)
    ref = OracleRun(img)
    kps, df = gpu_ctx.detect(img, desc_f32=True)
    assert final_ok(compare_final(kps, df, ref.final, ref.desc_f32))


@pytest.mark.slow
def test_gpu_8k_properties(gpu_ctx):
    """BASELINE config 5 (7680x4320, dense): size-independent properties."""
    img = synth_image(7680, 4320, 1, nblobs=1500000, smax=4.0, seed=42)
    kps, df = gpu_ctx.detect(img, desc_f32=True)
    c = gpu_ctx.counts()
    assert c["octaves"] == 11 and c["final_n"] == len(kps) > 100000
    # clean_keypoints order and uniqueness
    order = np.lexsort((-kps["octave"], kps["pori"], -kps["size"], kps["y"], kps["x"]))
    assert np.array_equal(order, np.arange(len(kps)))
    # keypoints inside the input image, orientations in [0, 2pi)
    assert kps["x"].min() >= 0 and kps["x"].max() < 7680
    assert kps["y"].min() >= 0 and kps["y"].max() < 4320
    assert kps["pori"].min() >= 0 and kps["pori"].max() < 2 * np.pi
    # descriptor floats: unit norm after the 0.2 clamp
    nrm = np.linalg.norm(df.astype(np.float64), axis=1)
    nrm = nrm[~np.isnan(nrm)]  # all-zero histograms give NaN (Appendix A.17)
    assert len(nrm) > 0.99 * len(kps) and np.all(np.abs(nrm - 1.0) < 1e-5)
    # next-octave base == decimated level `intervals` (sift.cpp:195-196)
    g3 = gpu_ctx.level(1, 3)
    g0n = gpu_ctx.level(2, 0)
    assert np.array_equal(g0n, g3[: g0n.shape[0] * 2: 2, : g0n.shape[1] * 2: 2])
    # each sampled extremum satisfies the cube condition on the pyramid
    ext = gpu_ctx.extrema()
    o = 3
    e = ext[ext["octave"] == o][:500]
    G = [gpu_ctx.level(o, lv) for lv in range(6)]
    D = [G[i + 1] - G[i] for i in range(5)]
    for x, y, z, _ in e:
        v = D[z][y, x]
        cube = np.stack([D[z + dz][y - 1:y + 2, x - 1:x + 2] for dz in (-1, 0, 1)])
        assert abs(v) > 1 and (v == cube.max() or v == cube.min())


# Every small-octave split against the oracle, level by level: the
# one-workgroup LDS-resident kernel from the default octave on (SIFT_LDS_PX
# 9088), from later octaves (2100, 600) or not at all (0: every octave by
# per-level launches). Odd and ragged shapes exercise partial tiles and
# clamped borders on every side.
@pytest.mark.parametrize("lds_px", ["9088", "2100", "600", "0"])
@pytest.mark.parametrize("shape", [(640, 360, 1), (333, 517, 3), (97, 61, 1)],
                         ids=["640x360", "333x517rgb", "97x61"])
def test_gpu_pyramid_paths_match_oracle(lds_px, shape):
    import os

    from sift_hip import Context

    os.environ["SIFT_LDS_PX"] = lds_px
    try:
        ctx = Context(0)
    finally:
        del os.environ["SIFT_LDS_PX"]
    try:
        w, h, c = shape
        img = synth_image(w, h, c, seed=w * 7 + h)
        ref = OracleRun(img)
        kps, df = ctx.detect(img, desc_f32=True)
        for o in range(ref.octaves):
            for lv in range(ref.levels):
                a, b = ctx.level(o, lv), ref.level(o, lv)
                assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (o, lv)
        assert np.array_equal(sort_extrema(ctx.extrema()), sort_extrema(ref.extrema))
        r = compare_final(kps, df, ref.final, ref.desc_f32)
        assert final_ok(r), r
    finally:
        ctx.close()


# The small octaves in flight (k_octaves_flow) against the oracle, level by
# level: the default split, every octave up to 4 Mpx in one launch with one
# workgroup (every dependency met in ticket order), 7 and 128 workgroups
# (tiles waiting on their neighbour bands, decimated planes across octaves),
# and the per-level launches (SIFT_FLOW=0).
@pytest.mark.parametrize("flow", [("1", "524288", "128"), ("1", "4194304", "1"),
                                  ("1", "4194304", "7"), ("1", "4194304", "128"),
                                  ("0", "0", "1")],
                         ids=["default", "all-1wg", "all-7wg", "all-128wg", "off"])
@pytest.mark.parametrize("shape", [(640, 360, 1), (333, 517, 3), (97, 61, 1)],
                         ids=["640x360", "333x517rgb", "97x61"])
def test_gpu_octaves_flow_match_oracle(flow, shape):
    import os

    from sift_hip import Context

    env = {"SIFT_FLOW": flow[0], "SIFT_FLOW_PX": flow[1], "SIFT_FLOW_WGS": flow[2],
           "SIFT_BATCH_PX_LOG2": "18"}
    os.environ.update(env)
    try:
        ctx = Context(0)
    finally:
        for k in env:
            del os.environ[k]
    try:
        w, h, c = shape
        img = synth_image(w, h, c, seed=w * 5 + h)
        ref = OracleRun(img)
        for rep in range(2):  # the second job reuses the slot's counters
            kps, df = ctx.detect(img, desc_f32=True)
            for o in range(ref.octaves):
                for lv in range(ref.levels):
                    a, b = ctx.level(o, lv), ref.level(o, lv)
                    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (rep, o, lv)
            assert np.array_equal(sort_extrema(ctx.extrema()), sort_extrema(ref.extrema))
            r = compare_final(kps, df, ref.final, ref.desc_f32)
            assert final_ok(r), r
    finally:
        ctx.close()


# Mid-sized octaves fused into one launch each (k_octave_fused: tiles with
# recomputed halos) against the oracle, level by level: the default split,
# every octave from octave 1 on with 32 x 32 or 16 x 16 tiles, without the
# LDS-resident octaves (so tiny octaves, down to a few pixels, are tiled
# too), other intervals (halos of 4 to 8 levels), and two jobs per context
# (the second reuses the slot). Ragged shapes give partial tiles and tiles
# whose halos are clipped on every side.
@pytest.mark.parametrize("fuse", [
    ({"SIFT_FUSE": "1"}, None),
    ({"SIFT_FUSE": "1", "SIFT_FUSE_PX": "4194304", "SIFT_FUSE_T32_PX": "0"}, None),
    ({"SIFT_FUSE": "1", "SIFT_FUSE_PX": "4194304", "SIFT_FUSE_T32_PX": "4194304",
      "SIFT_LDS_PX": "0"}, None),
    ({"SIFT_FUSE": "1", "SIFT_FUSE_PX": "4194304", "SIFT_LDS_PX": "0"}, {"intervals": 1}),
    ({"SIFT_FUSE": "1", "SIFT_FUSE_PX": "4194304", "SIFT_FUSE_T32_PX": "0"},
     {"intervals": 5, "init_sigma": 1.3}),
], ids=["default", "all-t32", "all-t16-nolds", "int1-nolds", "int5-t32"])
@pytest.mark.parametrize("shape", [(640, 360, 1), (333, 517, 3), (97, 61, 1)],
                         ids=["640x360", "333x517rgb", "97x61"])
def test_gpu_octave_fused_match_oracle(fuse, shape):
    import os

    from sift_hip import Context, SiftParams

    env, kw = fuse
    env = dict(env, SIFT_BATCH_PX_LOG2="18")
    os.environ.update(env)
    try:
        ctx = Context(0)
    finally:
        for k in env:
            del os.environ[k]
    try:
        w, h, c = shape
        img = synth_image(w, h, c, seed=w * 3 + h)
        p = SiftParams(**kw) if kw else None
        ref = OracleRun(img, p)
        for rep in range(2):
            kps, df = ctx.detect(img, p, desc_f32=True)
            for o in range(ref.octaves):
                for lv in range(ref.levels):
                    a, b = ctx.level(o, lv), ref.level(o, lv)
                    assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (rep, o, lv)
            assert np.array_equal(sort_extrema(ctx.extrema()), sort_extrema(ref.extrema))
            r = compare_final(kps, df, ref.final, ref.desc_f32)
            assert final_ok(r), r
    finally:
        ctx.close()


# The fused initial blur of a one-channel input (gray + bilinear x2 through
# the strip walk's ring of input rows, k_blur<R, 2, false, kSrcUpsample>) and
# the octave-0 pair walk on doubled planes of >= 4 Mpx, against the oracle:
# ragged strip and band counts (H0 not a multiple of the 32-row strips or the
# 64-row pair bands), both image borders, and a wider initial kernel
# (init_sigma 2.0: R = 5 instead of 4). (Round 6 measured the initial blur on
# the pair walk too, with the ring walking up or down: bit-exact here, but
# 63 vs 34 us per 1080p image, so it was removed.)
@pytest.mark.parametrize("case", [((1100, 1001), {}), ((1030, 1027), {"init_sigma": 2.0})],
                         ids=["1100x1001", "1030x1027-sigma2"])
def test_gpu_initial_blur_large_match_oracle(gpu_ctx, case):
    from sift_hip import SiftParams

    (w, h), kw = case
    img = synth_image(w, h, 1, seed=w + 7 * h)
    p = SiftParams(**kw) if kw else None
    ref = OracleRun(img, p)
    kps, df = gpu_ctx.detect(img, p, desc_f32=True)
    for o in range(2):
        for lv in range(ref.levels):
            a, b = gpu_ctx.level(o, lv), ref.level(o, lv)
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (o, lv)
    assert np.array_equal(sort_extrema(gpu_ctx.extrema()), sort_extrema(ref.extrema))
    r = compare_final(kps, df, ref.final, ref.desc_f32)
    assert final_ok(r), r


# The descriptor (k_descriptor_split, every per-sample operation in f64)
# against the 1080p golden and the stb-decoded photographs (natural
# gradients).
DESC_GOLDENS = [g for g in GOLDENS if g.name in ("synth_1920x1080", "image1",
                                                 "photo_cave01_00")]


@pytest.mark.parametrize("g", DESC_GOLDENS, ids=[g.name for g in DESC_GOLDENS])
def test_gpu_descriptor_f64_reference_precision(gpu_ctx, g):
    """Default descriptor: the reference's f64 sample math (sift.cpp:641-678)
    leaves only libm last bits and the summation order, so every u8 byte
    equals the reference's and the floats agree to f32 rounding."""
    kps, df = gpu_ctx.detect(g.input(), g.params(), desc_f32=True)
    r = compare_final(kps, df, g.final, g.desc_f32)
    print(g.name, r)
    assert final_ok(r), r
    assert r["desc_u8_mismatch"] == 0 and r["desc_f32_max"] <= DESC_F64_F32_TOL, r
