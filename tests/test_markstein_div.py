"""The projection divides several numerators by one norm with a shared reciprocal (gsm_device.h
div_many: y = RN(1/b), q = RN(a y), q' = RN(q + fma(-q, b, a) y)) and claims the result is bit for bit
IEEE a / b -- the oracle's division -- outside the ranges it hands back to the division.  Checked here
on the CPU (same IEEE single operations and fma) over random, signed-zero and fp16-valued pairs by
tools/exp/markstein_div.c; the GPU parity tests then compare whole frames."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_shared_reciprocal_division_is_correctly_rounded(tmp_path, mode):
    exe = tmp_path / "md"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(ROOT, "tools", "exp", "markstein_div.c"),
                    "-lm"], check=True)
    out = subprocess.run([str(exe), "3000000", str(mode)], check=True, capture_output=True, text=True).stdout
    assert out.strip().endswith("bad 0"), out
