"""Generate tests/golden/exp_h_table.npy: the correctly rounded fp16 value of e^x for
every fp16 bit pattern x, computed with Python's decimal module at 60 significant
digits and an exact nearest-even choice between the two fp16 neighbours.  This pins
the numeric contract's exp independently of both the C oracle and the
HIP library, which build their tables from a double-precision series.

Run: python tests/golden/make_exp_table.py
"""
import decimal
import os

import numpy as np

D = decimal.Decimal
decimal.getcontext().prec = 60


def half_value(bits: int) -> D:
    s = -1 if bits & 0x8000 else 1
    e = (bits >> 10) & 0x1F
    m = bits & 0x3FF
    if e == 0:
        return s * D(m) * D(2) ** -24
    return s * (D(1024 + m)) * D(2) ** (e - 25)


POS = [(b, half_value(b)) for b in range(0, 0x7C00)]  # all finite non-negative halves


def round_to_half(v: D) -> int:
    """Nearest-even fp16 (bits) for a non-negative decimal v."""
    if v >= D(65520):
        return 0x7C00
    lo, hi = 0, 0x7BFF
    while lo < hi:  # largest half <= v
        mid = (lo + hi + 1) // 2
        if POS[mid][1] <= v:
            lo = mid
        else:
            hi = mid - 1
    a = lo
    if POS[a][1] == v or a == 0x7BFF:
        return a
    b = a + 1
    da, db = v - POS[a][1], POS[b][1] - v
    if da < db:
        return a
    if db < da:
        return b
    return a if a % 2 == 0 else b


def main():
    out = np.zeros(65536, np.uint16)
    for bits in range(65536):
        e = (bits >> 10) & 0x1F
        m = bits & 0x3FF
        if e == 31:
            if m:
                out[bits] = 0x7E00 | (bits & 0x8000) | m  # NaN (payload kept, quiet bit set)
            else:
                out[bits] = 0 if bits & 0x8000 else 0x7C00  # e^-inf = 0, e^inf = inf
            continue
        x = half_value(bits)
        if x < -20:
            out[bits] = 0
            continue
        if x > 12:
            out[bits] = 0x7C00
            continue
        out[bits] = round_to_half(x.exp())
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "exp_h_table.npy")
    np.save(path, out)
    print("wrote", path)


if __name__ == "__main__":
    main()
