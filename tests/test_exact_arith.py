"""Exactness of the device arithmetic, checked on the host with
the same binary64 operation sequences the kernels use:

* tools/la_check.cpp: LeastAllocated floor((cap - req) * 100 / cap) as the
  truncation of fma(x, RN(1/cap), 2^-45), for every capacity < 2^44;
* tools/markstein_check.cpp: BalancedAllocation's IEEE quotient
  RN(a / b) = fma(fma(-b, q0, a), y, q0), q0 = RN(a y), y = RN(1/b).
"""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("src", ["la_check.cpp", "markstein_check.cpp"])
def test_exact_arith(tmp_path, src):
    exe = tmp_path / src.replace(".cpp", "")
    subprocess.run(["g++", "-O2", "-mfma", "-ffp-contract=off", str(ROOT / "tools" / src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout
