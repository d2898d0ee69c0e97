"""as_secs_f64 on the device divides the nanoseconds by 1e9 with a multiply and one FMA
correction instead of a general division (ruserf_amd/csrc/common.h).  It is exact because,
for every integer in [0, 1e9) -- the whole domain of Duration nanos -- the result equals the
correctly rounded quotient: checked here over all 1e9 values (a C loop, about 2 s)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_fma_division_by_1e9_exhaustive(tmp_path):
    exe = tmp_path / "div1e9"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(HERE, "div1e9_check.c"), "-lm"],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout
