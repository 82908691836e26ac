"""The C++ drop-in: the reference's unmodified main.cpp (+ its image.cpp /
image_io.cpp for stb I/O and drawing) linked against libsift_amd.so instead
of the reference's sift.cpp (oracle/Makefile target sift_amd_cli, built in
the build container where /root/reference exists; the binary travels)."""
import os
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
