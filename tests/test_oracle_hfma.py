"""The oracle's fused fp16 multiply-add (og_hfma, the blend's `C += c * w`) against an
exact rational restatement: round-to-nearest-even of a*b + c computed in Fractions."""
import os
import sys
from fractions import Fraction

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import oracle  # noqa: E402


def f16_value(bits: int) -> Fraction:
    return Fraction(float(np.array([bits], np.uint16).view(np.float16)[0]))


def round_f16(x: Fraction) -> int:
    """IEEE binary16 round-to-nearest-even of an exact rational (finite results only)."""
    sign = 0x8000 if x < 0 else 0
    a = -x if x < 0 else x
    if a == 0:
        return sign
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    q = Fraction(2) ** (max(e, -14) - 10)  # quantum of a's binade (subnormals: 2^-24)
    r = a / q
    n = r.numerator // r.denominator
    rem = r - n
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and n % 2 == 1):
        n += 1
    v = n * q
    if v >= 65520:
        return sign | 0x7C00
    bits = int(np.array([float(v)], np.float16).view(np.uint16)[0])
    return sign | bits


def finite_bits(rng, n, lo_exp=-24, hi_exp=8):
    """Random finite fp16 patterns biased to the blend's ranges, both signs, subnormals included."""
    mant = rng.integers(0, 1024, n)
    expo = rng.integers(0, 31, n)
    bits = (expo << 10) | mant
    bits[rng.random(n) < 0.2] &= 0x03FF  # subnormals
    bits[rng.random(n) < 0.2] |= 0x8000
    return bits.astype(np.int64)


def test_hfma_matches_exact_rounding():
    L = oracle.lib()
    rng = np.random.default_rng(7)
    a, b, c = (finite_bits(rng, 20000) for _ in range(3))
    # the blend's operands: colour / depth in [0, 1] or more, weights tiny to 0.99, accumulators small
    bad = []
    for x, y, z in zip(a.tolist(), b.tolist(), c.tolist()):
        exact = f16_value(x) * f16_value(y) + f16_value(z)
        if abs(exact) >= 65520:
            continue
        want = round_f16(exact)
        got = L.og_hfma(x, y, z)
        if got != want and not (exact == 0 and (got & 0x7FFF) == 0):
            bad.append((hex(x), hex(y), hex(z), hex(got), hex(want)))
    assert not bad, bad[:5]


@pytest.mark.parametrize("case", [
    (0x3C00, 0x3C00, 0x0000),  # 1*1 + 0
    (0x3C01, 0x3C01, 0x0000),  # product needs rounding
    (0x3C00, 0x3C00, 0x0001),  # 1 + smallest subnormal: below the half ulp
    (0x3C01, 0x3800, 0x0001),  # product exactly on a midpoint + tiny addend: rounds up
    (0x3C01, 0x3800, 0x8001),  # ... tiny negative addend: rounds down
    (0x3C03, 0x3800, 0x0000),  # exact midpoint, ties to even
])
def test_hfma_midpoints(case):
    L = oracle.lib()
    x, y, z = case
    assert L.og_hfma(x, y, z) == round_f16(f16_value(x) * f16_value(y) + f16_value(z))
