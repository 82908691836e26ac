"""The C++ drop-in: the reference's unmodified main.cpp (+ its image.cpp /
image_io.cpp for stb I/O and drawing) linked against libsift_amd.so instead
of the reference's sift.cpp (oracle/Makefile target sift_amd_cli, built in
the build container where /root/reference exists; the binary travels)."""
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "oracle", "_ref", "sift_amd_cli")


def _need_cli():
    if not os.path.exists(CLI):
        pytest.skip("sift_amd_cli not built (needs /root/reference: make -C oracle ref)")


def test_dropin_cli_links_against_libsift_amd():
    _need_cli()
    out = subprocess.run(["ldd", CLI], capture_output=True, text=True, check=True).stdout
    assert "libsift_amd.so" in out and "libsift_hip.so" in out
    syms = subprocess.run(["nm", "-D", "--undefined-only", CLI], capture_output=True,
                          text=True, check=True).stdout
    assert "detect_keypoints_and_descriptors" in syms and "match_keypoints" in syms


@pytest.mark.gpu
def test_dropin_cli_runs_reference_main(tmp_path):
    """`./sift img1 img2` (reference main.cpp:6-19) on the MI355X backend."""
    _need_cli()
    from PIL import Image as PILImage

    from golden_util import GOLDEN_DIR, Golden

    g = Golden(os.path.join(GOLDEN_DIR, "image1.npz"))
    a = g.input().astype(np.uint8)
    PILImage.fromarray(a).save(tmp_path / "a.png")
    PILImage.fromarray(np.ascontiguousarray(a[:, ::-1])).save(tmp_path / "b.png")
    r = subprocess.run([CLI, "a.png", "b.png"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "keypoints.png").stat().st_size > 0
    assert (tmp_path / "matches.png").stat().st_size > 0


@pytest.mark.gpu
def test_dropin_cli_outputs_equal_reference_cli(tmp_path):
    """`./sift image1.jpg image2.jpg` on the MI355X backend leaves the same
    keypoints.png (the last detect's, sift.cpp:765-768) and matches.png
    (sift.cpp:850-876) as the reference CLI, byte for byte (fixtures:
    tests/golden/cli_outputs.json, made by make_goldens.py --cli from the
    reference's own main.cpp + sift.cpp, copy-fixed build)."""
    _need_cli()
    gdir = os.path.join(ROOT, "tests", "golden")
    want = json.load(open(os.path.join(gdir, "cli_outputs.json")))
    for n, h in want["inputs"].items():
        shutil.copyfile(os.path.join(gdir, n), tmp_path / n)
        assert hashlib.sha256((tmp_path / n).read_bytes()).hexdigest() == h
    r = subprocess.run([CLI, "cli_image1.jpg", "cli_image2.jpg"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    for f in ("keypoints.png", "matches.png"):
        assert hashlib.sha256((tmp_path / f).read_bytes()).hexdigest() == want[f], f
