"""Accuracy of regcm_amd/csrc/fastmath.hpp (the fdlibm-class log/exp the dyn kernels use for
the hypsometric/PGF logs and the vadv x**y), measured on the host against long-double libm:
max error below 1 ulp for log and exp, and for x**y over the pressure/humidity ratios of the
step (the same header is compiled into the gfx950 kernels)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_fastmath_ulp_error(tmp_path):
    exe = tmp_path / "fmcheck"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-o", str(exe),
                    os.path.join(ROOT, "tests", "fastmath", "fastmath_check.cpp")], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    elog, eexp, epow = map(float, out)
    assert elog < 1.0 and eexp < 1.0
    assert epow < 1.5


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_div_by_is_ieee_division(tmp_path):
    """rcm::div_by (x / y from a hoisted 1 / y: one product and two FMAs, Markstein's
    correction) returns the bits of the IEEE division x / y; the split-step kernels use it for
    their loop-invariant denominators and stay bit-identical to the oracle's divisions."""
    exe = tmp_path / "divcheck"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-o", str(exe),
                    os.path.join(ROOT, "tests", "fastmath", "divby_check.cpp")], check=True)
    n, bad = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert n == 10000000 and bad == 0
