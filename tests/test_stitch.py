"""Stitching consumer: stitch-graph parsing, GPU RANSAC
and GPU compositing against the oracle restatement (oracle/stitch_cpu.cpp),
and an end-to-end stitch of a slice of the reference's CAVE-04_times_square
dataset (tests/golden/stitch/, tests/golden/make_stitch_fixture.py).

Parity: PINNED to the oracle only — bit-exact hypothesis scores, models,
inlier masks and canvases. Against the reference it is UNPINNED: the
reference's stitching notebook (stitching/sift_stitch.ipynb) is absent
(.MISSING_LARGE_BLOBS:3), so there is no reference output; ground-truth
properties (known synthetic homographies) stand in for it.
"""
import glob
import os

import numpy as np
import pytest

from oracle_bind import oracle_ransac_homography, oracle_ransac_scores, oracle_warp_blend
from sift_stitch import (PairResult, StitchGraph, canvas_for, compose, load_dataset,
                         read_stitch_graph)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "stitch")
REF_GRAPHS = sorted(glob.glob("/root/reference/stitching/collection/Dataset/*/*-STITCH-GRAPH.txt"))


def _apply(H, p):
    q = np.c_[p, np.ones(len(p))] @ H.T
    return q[:, :2] / q[:, 2:]


def _synthetic_pairs(n=600, outlier_frac=0.3, seed=7):
    rng = np.random.default_rng(seed)
    H = np.array([[0.98, -0.05, 40.0], [0.04, 1.01, -25.0], [2e-5, -1e-5, 1.0]])
    src = rng.uniform(0, 640, size=(n, 2))
    dst = _apply(H, src) + rng.normal(0, 0.3, size=(n, 2))
    k = int(n * outlier_frac)
    dst[:k] = rng.uniform(0, 640, size=(k, 2))
    return H, src, dst, k


# ---- host logic and the oracle (CPU) ---------------------------------------
def test_read_stitch_graph_fixture():
    g = read_stitch_graph(os.path.join(FIX, "cave04_sub-STITCH-GRAPH.txt"))
    assert (g.center, g.rotation, g.count) == (2, 0.0, 5)
    assert g.pairs() == [(0, 1), (1, 2), (2, 3), (3, 4)]


@pytest.mark.skipif(not REF_GRAPHS, reason="reference checkout not present")
@pytest.mark.parametrize("path", REF_GRAPHS, ids=[os.path.basename(p) for p in REF_GRAPHS])
def test_read_reference_stitch_graphs(path):
    g = read_stitch_graph(path)
    n_lines = sum(1 for ln in open(path) if "matching_graph_image_edges-" in ln)
    assert len(g.edges) == n_lines and 0 <= g.center < g.count
    assert all(0 <= j < g.count for js in g.edges.values() for j in js)


def test_oracle_ransac_recovers_known_homography():
    H, src, dst, k = _synthetic_pairs()
    Hest, mask, n_in = oracle_ransac_homography(src, dst)
    assert n_in >= 0.95 * (len(src) - k)
    assert mask[:k].mean() < 0.02
    err = np.linalg.norm(_apply(Hest, src[k:]) - _apply(H, src[k:]), axis=1)
    assert err.max() < 0.5


def test_oracle_ransac_degenerate_points_have_no_model():
    src = np.c_[np.arange(20.0), 2.0 * np.arange(20.0)]  # collinear
    sc = oracle_ransac_scores(src, src + 5.0, n_hyp=64)
    assert (sc == -1).all()
    H, mask, n_in = oracle_ransac_homography(src, src + 5.0, n_hyp=64)
    assert n_in == 0 and np.array_equal(H, np.eye(3))


def test_oracle_warp_identity_reproduces_image():
    rng = np.random.default_rng(3)
    im = rng.integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    out = oracle_warp_blend([im], [np.eye(3)], 53, 37)
    assert np.array_equal(out, im)


def test_compose_and_canvas_chain():
    g = StitchGraph(center=1, rotation=0.0, count=3, edges={0: [1], 1: [2]})
    T01 = np.array([[1, 0, 100.0], [0, 1, 0], [0, 0, 1]])   # image 1 -> image 0
    T12 = np.array([[1, 0, 100.0], [0, 1, 10], [0, 0, 1]])  # image 2 -> image 1
    pairs = [PairResult(0, 1, T01, 50, 40), PairResult(1, 2, T12, 50, 40)]
    Hs = compose(g, pairs, 3)
    assert np.allclose(Hs[1], np.eye(3))
    assert np.allclose(Hs[2], T12)
    assert np.allclose(Hs[0], np.linalg.inv(T01))
    ims = [np.zeros((50, 200, 3), np.uint8)] * 3
    T, W, H = canvas_for(ims, Hs)
    assert (W, H) == (200 + 200, 50 + 10)
    assert np.allclose(T[:2, 2], [100.0, 0.0])


def test_canvas_clips_around_the_centre_image():
    # a 6000-px-wide centre image far from the origin keeps its whole extent
    # when a neighbour flies off; the clip window is centred on it
    ims = [np.zeros((100, 6000, 3), np.uint8), np.zeros((100, 100, 3), np.uint8)]
    far = np.array([[1, 0, 1e6], [0, 1, 0], [0, 0, 1.0]])
    Hs = {0: np.array([[1, 0, 20000.0], [0, 1, 0], [0, 0, 1]]), 1: far}
    T, W, H = canvas_for(ims, Hs, max_side=8192)
    assert W <= 8192 and H == 100
    lo = -T[0, 2]
    assert lo <= 20000 and lo + W - 1 >= 20000 + 5999   # centre image fully inside
    # every image (the centre included) projected behind the camera: the
    # centre image's own box, no exception
    behind = np.array([[1, 0, 0], [0, 1, 0], [0, 0, -1.0]])
    T, W, H = canvas_for(ims, {0: behind, 1: behind})
    assert (W, H) == (6000, 100) and np.allclose(T[:2, 2], [0.0, 0.0])


# ---- GPU (HIP through the C-ABI) --------------------------------------------
@pytest.mark.gpu
def test_gpu_ransac_scores_and_model_equal_oracle(gpu_ctx):
    H, src, dst, k = _synthetic_pairs()
    for kw in (dict(), dict(n_hyp=1000, threshold=1.5, seed=99, refine_iters=0)):
        sg = gpu_ctx.ransac_scores(src, dst, **{k2: v for k2, v in kw.items()
                                                if k2 != "refine_iters"})
        so = oracle_ransac_scores(src, dst, **{k2: v for k2, v in kw.items()
                                               if k2 != "refine_iters"})
        assert np.array_equal(sg, so)
        Hg, mg, ng = gpu_ctx.ransac_homography(src, dst, **kw)
        Ho, mo, no = oracle_ransac_homography(src, dst, **kw)
        assert ng == no and np.array_equal(mg, mo)
        assert np.array_equal(Hg.view(np.uint64), Ho.view(np.uint64))
        if kw.get("refine_iters", 2):  # the refitted model is close to the truth
            err = np.linalg.norm(_apply(Hg, src[k:]) - _apply(H, src[k:]), axis=1)
            assert err.max() < 0.5


@pytest.mark.gpu
def test_gpu_ransac_edges(gpu_ctx):
    src = np.c_[np.arange(20.0), 2.0 * np.arange(20.0)]
    assert (gpu_ctx.ransac_scores(src, src + 5.0, n_hyp=64) == -1).all()
    H, mask, n_in = gpu_ctx.ransac_homography(src, src + 5.0, n_hyp=64)
    assert n_in == 0 and np.array_equal(H, np.eye(3))
    with pytest.raises(RuntimeError):
        gpu_ctx.ransac_homography(src[:3], src[:3])
    # exactly four pairs: the one model fits them all
    sq = np.array([[0, 0], [10, 0], [10, 10], [0, 10.0]])
    H, mask, n_in = gpu_ctx.ransac_homography(sq, sq * 2 + 3, n_hyp=8)
    assert n_in == 4 and np.allclose(_apply(H, sq), sq * 2 + 3)


@pytest.mark.gpu
def test_gpu_warp_blend_equals_oracle(gpu_ctx):
    rng = np.random.default_rng(11)
    ims = [rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
           for (h, w) in ((60, 80), (45, 70), (50, 50))]
    Hs = []
    for t in range(3):
        A = np.eye(3)
        A[:2, 2] = [-15.0 * t, -7.0 * t]
        A[0, 1] = 0.05 * t
        A[2, :2] = [1e-4 * t, -2e-4 * t]
        Hs.append(A)
    for c in (3, 1):
        cims = ims if c == 3 else [im[:, :, 0] for im in ims]
        g = gpu_ctx.warp_blend(cims, Hs, 150, 110)
        o = oracle_warp_blend(cims, Hs, 150, 110)
        assert np.array_equal(g, o)
    assert g.any()


@pytest.mark.gpu
def test_gpu_stitch_dataset_fixture(gpu_ctx):
    """Five CAVE-04_times_square images along their stitch graph: every
    image placed, every edge's GPU RANSAC model equal to the oracle's on the
    same GPU matches, the inliers reprojected within the threshold."""
    from sift_stitch import keypoint_xy, stitch

    graph, images = load_dataset(FIX)
    assert len(images) == 5
    res = stitch(gpu_ctx, images, graph)
    assert res.placed == [0, 1, 2, 3, 4]
    assert len(res.pairs) == 4
    for p in res.pairs:
        assert p.inliers >= 30 and p.inliers >= 0.3 * p.matches, (p.i, p.j, p.matches, p.inliers)
        m = gpu_ctx.match(res.keypoints[p.j], res.keypoints[p.i], 0.75)
        src = keypoint_xy(res.keypoints[p.j])[m["i1"]]
        dst = keypoint_xy(res.keypoints[p.i])[m["i2"]]
        Ho, mo, no = oracle_ransac_homography(src, dst)
        assert no == p.inliers
        assert np.array_equal(Ho.view(np.uint64), p.H.view(np.uint64))
        e = np.linalg.norm(_apply(p.H, src[mo]) - dst[mo], axis=1)
        assert e.max() < 3.0
    h, w = res.panorama.shape[:2]
    assert w >= 640 and h >= 480 and w * h <= 8192 * 8192
    assert (res.panorama.sum(axis=2) > 0).mean() > 0.3
