"""GPU: the descriptor's f64 sqrt / atan2 / exp (sift-project_amd/csrc/
sift_math64.h) against the device's correctly rounded sqrt, ocml's atan2 /
exp and the host's glibc, on the argument ranges of the descriptor's sample
math (reference src/sift.cpp:660-672). tools/math64_check is built by
__graft_entry__.build().

Bars: sqrt bit-identical to the correctly rounded sqrt; atan2 and exp within
1 ulp of glibc (glibc itself is not correctly rounded in ~0.1 % of calls,
DESIGN §2), differing from glibc in a small fraction of arguments.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "math64_check")


def test_gpu_math64_accuracy():
    assert os.path.exists(BIN), "tools/math64_check not built (__graft_entry__.build())"
    out = subprocess.run([BIN, str(1 << 22)], capture_output=True, text=True, timeout=120,
                         check=True).stdout
    res = {}
    for line in out.splitlines():
        name, *kv = line.split()
        res[name] = {k: float(v) for k, v in (x.split("=") for x in kv)}
    print(res)
    assert set(res) == {"sqrt", "atan2", "exp", "atan2_f32", "atan2_tiny"}
    # gradients below the f32 normal range / subnormal (never from image
    # data): the out-of-line ocml fallback, a few ulp from glibc at worst
    assert res["atan2_tiny"]["ulp_max_dev"] == 0 and res["atan2_tiny"]["ulp_max_glibc"] <= 4
    # orientation bins: f32 atan2 well inside k_orient_wave's guard band
    # (nb * 3e-6 in bin units, i.e. 5e-4 rad at 36 bins)
    assert res["atan2_f32"]["abs_err_max_rad"] < 1e-6
    assert res["sqrt"]["ulp_max_dev"] == 0 and res["sqrt"]["ulp_max_glibc"] == 0
    for fn in ("atan2", "exp"):
        assert res[fn]["ulp_max_glibc"] <= 1, (fn, res[fn])
        assert res[fn]["diff_frac_glibc"] < 0.25, (fn, res[fn])
