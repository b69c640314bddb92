"""Derive the Float64 values of Julia's `range(-π, π, 8)` (src/Modulation.jl:360).

TEST/ORACLE TOOL.  Replays Base.twiceprecision `_linspace(start, stop, len)` for Float64
(the rational fast path `rat()` fails for π: its 2^24-bounded convergent 5419351/1725033 does
not round back to Float64(π)), then `unsafe_getindex` of the resulting StepRangeLen.
Python floats are IEEE binary64, so the arithmetic below is bit-identical to Julia's.
"""
import math
import struct
from fractions import Fraction


def truncbits(x, nb):
    u = struct.unpack("<Q", struct.pack("<d", x))[0]
    u &= (0xFFFFFFFFFFFFFFFF << nb) & 0xFFFFFFFFFFFFFFFF
    return struct.unpack("<d", struct.pack("<Q", u))[0]


def add12(x, y):
    if abs(y) > abs(x):
        x, y = y, x
    h = x + y
    return h, (x - h) + y


def julia_rat(x):
    y = x
    a = d = 1
    b = c = 0
    m = 16777216  # maxintfloat(Float32, Int)
    while abs(y) <= m:
        f = math.trunc(y)
        y -= f
        a, c = f * a + c, a
        b, d = f * b + d, b
        if max(abs(a), abs(b)) > m:
            return c, d
        if float(a) / float(b) == x:
            break
        y = 1.0 / y
    return a, b


def julia_range(start, stop, n):
    sn, sd = julia_rat(start)
    en, ed = julia_rat(stop)
    den = sd * ed // math.gcd(sd, ed)
    if den and abs(den * start) <= 2**53 and abs(den * stop) <= 2**53:
        sn2, en2 = round(den * start), round(den * stop)
        if sn2 / den == start and en2 / den == stop:
            raise NotImplementedError("rational path not needed for ±π")
    delta = stop - start
    tmin = -(start / delta)
    imin = round(tmin * (n - 1) + 1)  # Python round = ties-to-even like Julia round
    assert 1 < imin < n
    t = (imin - 1) / (n - 1)
    ref = (1 - t) * start + t * stop
    step = (ref - start) / (imin - 1) if imin - 1 < n - imin else (stop - ref) / (n - imin)
    nb = min(27, math.ceil(math.log2(max(imin - 1, n - imin))))
    step_hi = truncbits(step, nb)
    x1_hi, x1_lo = add12((1 - imin) * step_hi, ref)
    x2_hi, x2_lo = add12((n - imin) * step_hi, ref)
    a = (start - x1_hi) - x1_lo
    b = (stop - x2_hi) - x2_lo
    step_lo = (b - a) / (n - 1)
    ref_lo = a - (1 - imin) * step_lo
    out = []
    for i in range(1, n + 1):
        u = i - imin
        shift_hi, shift_lo = u * step_hi, u * step_lo
        x_hi, x_lo = add12(ref, shift_hi)
        out.append(x_hi + (x_lo + (shift_lo + ref_lo)))
    return out


if __name__ == "__main__":
    vals = julia_range(-math.pi, math.pi, 8)
    for k, v in enumerate(vals):
        exact = float(Fraction(math.pi) * (2 * k - 7) / 7)
        print(f"{k}: {v!r:24} {v.hex():26} naive-correctly-rounded={exact.hex()} same={v == exact}")
