"""CPU: pin the oracle restatement to the reference's golden vectors.

The goldens were produced by the reference itself (src/sift.cpp compiled from
/root/reference by oracle/Makefile, tests/golden/make_goldens.py). The oracle
must reproduce them bit for bit: pyramid level hashes, the extrema set, the
final keypoint records (x, y, octave, layer, size, pori, desc) and the
normalised descriptor floats.
"""
import numpy as np
import pytest

from golden_util import all_goldens, sha256_array
from oracle_bind import OracleRun
from parity import sort_extrema
from sift_hip import EXT_DTYPE, SiftParams, synth_image

GOLDENS = all_goldens(kinds=("small", "medium"))


@pytest.mark.parametrize("g", GOLDENS, ids=[g.name for g in GOLDENS])
def test_oracle_matches_reference_golden(g):
    img = g.input()  # also checks the deterministic generator's sha256
    run = OracleRun(img, g.params())
    m = g.meta
    assert run.octaves == m["octaves"]
    assert len(run.extrema) == m["extrema"]
    assert len(run.refined) == m["refined"]
    assert len(run.oriented) == m["oriented"]
    assert len(run.final) == m["final"]
    # final records, byte for byte (pori and desc included: same glibc)
    assert run.final.tobytes() == g.final.tobytes()
    assert np.array_equal(run.desc_f32.view(np.uint32), g.desc_f32.view(np.uint32))
    # extrema set
    ge = np.zeros(len(g.extrema), dtype=EXT_DTYPE)
    for i, f in enumerate(("x", "y", "z", "octave")):
        ge[f] = g.extrema[:, i]
    assert np.array_equal(sort_extrema(run.extrema), sort_extrema(ge))
    # every Gaussian level
    if g.pyr_sha256 is not None:
        hashes = g.level_hashes()
        for o in range(run.octaves):
            for lv in range(run.levels):
                assert sha256_array(run.level(o, lv)) == hashes[o][lv], (o, lv)


def test_synth_generator_is_deterministic():
    a = synth_image(97, 53, 1, seed=5)
    b = synth_image(97, 53, 1, seed=5)
    c = synth_image(97, 53, 1, seed=6)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a.min() >= 0 and a.max() <= 255 and np.all(a == np.round(a))
    rgb = synth_image(31, 17, 3, seed=5)
    assert rgb.shape == (17, 31, 3)


def test_oracle_rejects_degenerate_inputs():
    with pytest.raises(RuntimeError):
        OracleRun(np.zeros((1, 1)))  # min(W0,H0)/3 == 0 -> log2(0) in the reference
    with pytest.raises(RuntimeError):
        OracleRun(np.zeros((8, 8, 2)))  # 2 channels: reference reads past the pixel


def test_oracle_parameter_variants_run():
    img = synth_image(120, 90, 1, seed=9)
    for p in (SiftParams(window_size=5), SiftParams(num_bins=72, peak_ratio=0.5),
              SiftParams(contrast_threshold=0.02, eigen_ratio=5.0),
              SiftParams(ori_sigma_factor=2.0, desc_scale_factor=4.0)):
        run = OracleRun(img, p)
        assert len(run.final) >= 0
        if len(run.final):
            k = run.final
            order = np.lexsort((-k["octave"], k["pori"], -k["size"], k["y"], k["x"]))
            assert np.array_equal(order, np.arange(len(k)))


def test_parameter_cases_are_pinned_to_the_reference():
    """Every stagewise GPU case (tests/test_gpu_parity.py CASES) has a golden
    produced by the reference with the same input and all sift.hh:65-71
    arguments (tests/golden/case_<name>.npz, checked above bit for bit)."""
    import zlib

    from test_gpu_parity import CASES

    by_name = {g.name: g for g in GOLDENS}
    for name, w, h, c, p in CASES:
        g = by_name["case_" + name]
        m = g.meta
        assert (m["w"], m["h"], m["c"], m["seed"]) == (w, h, c, zlib.crc32(name.encode()) & 0xFFFF)
        assert g.params() == p, name


@pytest.mark.parametrize("g", all_goldens(kinds=("big",)), ids=lambda g: g.name)
def test_big_goldens_full_arrays_consistent(g):
    """Configs 3 and 5 keep every keypoint's u8 descriptor and pori (the
    GPU test compares all of them); they must agree with the 64 full records
    and the descriptor-float samples the same reference run wrote."""
    desc, pori = g.full_desc_u8(), g.full_pori()
    n = g.meta["final"]
    assert desc.shape == (n, 128) and pori.shape == (n,)
    assert np.array_equal(desc[g.sample_idx], g.final["desc"])
    assert np.array_equal(pori[g.sample_idx].view(np.uint64), g.final["pori"].view(np.uint64))
    sidx, sdf = g.strat_sample()
    assert len(sidx) == min(4096, n) and np.all(np.diff(sidx) > 0)
    # quantisation of the floats the reference wrote (sift.cpp:600-601)
    q = np.minimum(np.floor(512.0 * sdf.astype(np.float64)), 255)
    assert np.mean(np.abs(q - desc[sidx]) <= 1) == 1.0
    assert np.all((pori >= 0) & (pori < 2 * np.pi))
