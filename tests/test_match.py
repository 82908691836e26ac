"""Matcher parity: the GPU 2-NN ratio-test matcher
(sift_match.hip, C-ABI sift_hip_match) against the reference match_keypoints
(src/sift.cpp:783-815).

tests/golden/match_cases.npz holds the reference's own outputs (made by
tests/golden/make_goldens.py --match through oracle/_ref/ref_harness): the
stitching image pair at the CLI's ratio, tie-heavy descriptors at three
ratios and the n2 == 1 case. The CPU test pins the oracle to them; the GPU
tests require exact equality (indices bit-exact, distances bit-exact: the
distance is sqrt of an exact integer)."""
import os

import numpy as np
import pytest

from oracle_bind import oracle_match
from sift_hip import KP_DTYPE, MATCH_DTYPE

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "match_cases.npz"))
NAMES = [str(n) for n in G["names"]]


def records(desc):
    k = np.zeros(len(desc), dtype=KP_DTYPE)
    k["x"] = np.arange(len(desc))
    k["desc"] = desc
    return k


def case(name):
    return (records(G[name + "__desc1"]), records(G[name + "__desc2"]),
            float(G[name + "__ratio"]), G[name + "__matches"])


def same(got, want):
    assert len(got) == len(want)
    assert np.array_equal(got["i1"].astype(np.int64), want["i1"].astype(np.int64))
    assert np.array_equal(got["i2"].astype(np.int64), want["i2"].astype(np.int64))
    assert np.array_equal(got["distance"], want["distance"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_match_reference_golden(name):
    k1, k2, r, want = case(name)
    same(oracle_match(k1, k2, r), want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_match_reference_golden(gpu_ctx, name):
    k1, k2, r, want = case(name)
    same(gpu_ctx.match(k1, k2, r), want)


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,lo,hi,ratio", [
    (1, 1, 0, 256, 0.75), (31, 33, 0, 256, 0.75), (100, 1000, 0, 4, 1.0),
    (2000, 3000, 0, 256, 0.8), (65, 64, 250, 256, 2.0), (3, 2, 0, 1, 0.75),
])
def test_gpu_match_vs_oracle(gpu_ctx, n1, n2, lo, hi, ratio):
    rng = np.random.default_rng(n1 * 7 + n2)
    k1 = records(rng.integers(lo, hi, size=(n1, 128), dtype=np.uint8))
    k2 = records(rng.integers(lo, hi, size=(n2, 128), dtype=np.uint8))
    same(gpu_ctx.match(k1, k2, ratio), oracle_match(k1, k2, ratio))


@pytest.mark.gpu
def test_gpu_match_edges_and_device_input(gpu_ctx):
    import torch
    k = records(np.random.default_rng(1).integers(0, 256, size=(50, 128), dtype=np.uint8))
    empty = np.zeros(0, dtype=KP_DTYPE)
    assert len(gpu_ctx.match(k, empty)) == 0
    assert len(gpu_ctx.match(empty, k)) == 0
    # a keypoint matched against itself: distance 0 to itself, ratio test passes
    m = gpu_ctx.match(k, k, 0.75)
    assert np.array_equal(m["i1"], np.arange(50)) and np.array_equal(m["i2"], np.arange(50))
    assert np.all(m["distance"] == 0.0)
    d1 = torch.from_numpy(k.view(np.uint8).copy()).cuda()
    got = gpu_ctx.match_device(d1.data_ptr(), 50, d1.data_ptr(), 50, 0.75)
    same(got, m)


@pytest.mark.gpu
def test_gpu_match_detected_keypoints(gpu_ctx):
    """Matcher on detector output: two synthetic 640x480 images sharing content."""
    from sift_hip import synth_image
    a = gpu_ctx.detect(synth_image(640, 480, seed=3))[0]
    b = gpu_ctx.detect(synth_image(640, 480, seed=3)[:, 8:])[0]
    same(gpu_ctx.match(a, b, 0.75), oracle_match(a, b, 0.75))
    assert MATCH_DTYPE.itemsize == 16
