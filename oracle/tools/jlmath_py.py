#!/usr/bin/env python3
"""An independent second restatement of Julia Base's Float64 sin / cos / sincos / rem_pio2 /
atan / atan(y, x) / hypot, in plain Python — TEST INFRASTRUCTURE ONLY.

Why: the oracle (oracle/demod_oracle.c) and the device share one C restatement of these
functions (gppupildemodulation.jl_amd/csrc/gpd_jlmath.h), so "the exact path equals the oracle
bit for bit" shows that both run the same source, not that the source is Julia's.  This module
is written again from the published algorithms, without the C header: Julia's
base/special/trig.jl (sin/cos/sincos kernels, atan, atan(y, x)), base/special/rem_pio2.jl
(two-constant and extended Cody–Waite reduction, the medium-precision Payne–Hanek reduction with
the 1/(2π) table and `fromfraction`) and base/math.jl (hypot), which restate FreeBSD msun
(k_sin.c, k_cos.c, e_rem_pio2.c, s_atan.c, e_atan2.c) with Julia's `muladd` (one rounding, as
on hardware with FMA) in the `@horner` polynomials.  Coefficients are taken as msun's IEEE bit
patterns; the 1/(2π) words come from oracle/tools/inv2pi.py (Machin's formula).

Arithmetic: Python floats are IEEE binary64 with round-to-nearest-even for + − × / and
math.sqrt; a fused multiply-add is evaluated exactly with Fraction and rounded once.
tests/test_jlmath_independent.py compares this module with the shared restatement bit for bit.
Julia itself is not available here, so agreement pins the C header against a second
transcription of the same published source, not against a Julia run.
"""
from __future__ import annotations

import math
import os
import struct
import sys
from fractions import Fraction

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import inv2pi  # noqa: E402

M64 = (1 << 64) - 1
M128 = (1 << 128) - 1


def _bits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def _f(u: int) -> float:
    return struct.unpack("<d", struct.pack("<Q", u & M64))[0]


def _poshighword(x: float) -> int:
    return (_bits(x) >> 32) & 0x7FFFFFFF


def _highword(x: float) -> int:
    return _bits(x) >> 32


def fma(a: float, b: float, c: float) -> float:
    """a·b + c rounded once (round to nearest, ties to even)."""
    if not (math.isfinite(a) and math.isfinite(b) and math.isfinite(c)):
        return a * b + c
    if a == 0.0 or b == 0.0:
        return a * b + c  # exact zero product: IEEE signed-zero rules of the addition
    r = Fraction(a) * Fraction(b) + Fraction(c)
    if r == 0:
        return 0.0  # exact cancellation of a nonzero product: +0 under round-to-nearest
    return float(r)  # int/int true division is correctly rounded


def horner(x: float, *c: float) -> float:
    """Julia's @horner(x, c0, c1, ..., cn) = muladd(x, muladd(x, ..., c1), c0)."""
    acc = c[-1]
    for k in range(len(c) - 2, -1, -1):
        acc = fma(x, acc, c[k])
    return acc


# ---- msun coefficients (k_sin.c S1..S6, k_cos.c C1..C6), as bit patterns ---------------------
DS1, DS2, DS3, DS4, DS5, DS6 = (_f(u) for u in (
    0xBFC5555555555549, 0x3F8111111110F8A6, 0xBF2A01A019C161D5,
    0x3EC71DE357B1FE7D, 0xBE5AE5E68A2B9CEB, 0x3DE5D93A5ACFD57C))
DC1, DC2, DC3, DC4, DC5, DC6 = (_f(u) for u in (
    0x3FA555555555554C, 0xBF56C16C16C15177, 0x3EFA01A019CB1590,
    0xBE927E4F809C52AD, 0x3E21EE9EBDB4B1C4, 0xBDA8FAE9BE8838D4))
PI = _f(0x400921FB54442D18)


def sin_kernel(y: float) -> float:
    """|y| ≤ π/4, no tail (Julia sin_kernel(::Float64))."""
    y2 = y * y
    y4 = y2 * y2
    r = horner(y2, DS2, DS3, DS4) + y2 * y4 * horner(y2, DS5, DS6)
    y3 = y2 * y
    return y + y3 * (DS1 + y2 * r)


def sin_kernel_dd(hi: float, lo: float) -> float:
    """sin_kernel(::DoubleFloat64), the reduced argument hi + lo."""
    y2 = hi * hi
    y4 = y2 * y2
    r = horner(y2, DS2, DS3, DS4) + y2 * y4 * horner(y2, DS5, DS6)
    y3 = y2 * hi
    return hi - ((y2 * (0.5 * lo - y3 * r) - lo) - y3 * DS1)


def cos_kernel_dd(hi: float, lo: float) -> float:
    y2 = hi * hi
    y4 = y2 * y2
    r = y2 * horner(y2, DC1, DC2, DC3) + y4 * y4 * horner(y2, DC4, DC5, DC6)
    half_y2 = 0.5 * y2
    w = 1.0 - half_y2
    return w + (((1.0 - w) - half_y2) + (y2 * r - hi * lo))


# ---- argument reduction (base/special/rem_pio2.jl) --------------------------------------------
PIO2_1 = _f(0x3FF921FB54400000)
PIO2_1T = _f(0x3DD0B4611A626331)
PIO2_2 = _f(0x3DD0B4611A600000)
PIO2_2T = _f(0x3BA3198A2E037073)
PIO2_3 = _f(0x3BA3198A2E000000)
PIO2_3T = _f(0x397B839A252049C1)
INVPIO2 = _f(0x3FE45F306DC9C883)


def _cw_2c(x: float, fn: float, n: int):
    z = fma(-fn, PIO2_1, x)
    y1 = fma(-fn, PIO2_1T, z)
    y2 = fma(-fn, PIO2_1T, z - y1)
    return n, y1, y2


def _cw_ext(x: float, xhp: int):
    fn = float(round(x * INVPIO2))  # Python round(): ties to even, like Julia's round
    r = fma(-fn, PIO2_1, x)
    w = fn * PIO2_1T
    j = xhp >> 20
    y1 = r - w
    i = j - ((_highword(y1) >> 20) & 0x7FF)
    if i > 16:
        t = r
        w = fn * PIO2_2
        r = t - w
        w = fma(fn, PIO2_2T, -((t - r) - w))
        y1 = r - w
        i = j - ((_highword(y1) >> 20) & 0x7FF)
        if i > 49:
            t = r
            w = fn * PIO2_3
            r = t - w
            w = fma(fn, PIO2_3T, -((t - r) - w))
            y1 = r - w
    y2 = (r - y1) - w
    return int(fn), y1, y2


_INV2PI = inv2pi.inv2pi_words(24)
# π/2 for the last step of Payne–Hanek: the double nearest π/2, and a head of 26 significant bits
# (its products with the 26-bit head of the fraction are exact) plus the double nearest the rest
_PI_EXACT = Fraction(inv2pi.pi_fixed(400), 1 << 400)
PIO2 = float(_PI_EXACT / 2)
PIO2_HI = float(Fraction(round(_PI_EXACT / 2 * (1 << 25)), 1 << 25))
PIO2_LO = float(_PI_EXACT / 2 - Fraction(PIO2_HI))


def _fromfraction(f: int):
    """A signed 128-bit fixed-point fraction (units 2^-128) as a 26-bit head + 53-bit tail."""
    if f == 0:
        return 0.0, 0.0
    s = (1 << 63) if f < 0 else 0
    x = abs(f)
    n1 = x.bit_length()
    m1 = ((x >> (n1 - 26)) & M64) << 27
    d1 = ((n1 - 128 + 1021) & M64) << 52
    z1 = _f(s | ((d1 + m1) & M64))
    x2 = x - (m1 << (n1 - 53)) if n1 >= 53 else x - (m1 >> (53 - n1))
    if x2 == 0:
        return z1, 0.0
    n2 = x2.bit_length()
    m2 = (x2 >> (n2 - 53)) if n2 >= 53 else (x2 << (53 - n2))
    d2 = ((n2 - 128 + 1021) & M64) << 52
    z2 = _f(s | ((d2 + (m2 & M64)) & M64))
    return z1, z2


def _payne_hanek(x: float):
    u = _bits(x)
    X = (u & ((1 << 52) - 1)) | (1 << 52)
    k = ((u >> 52) & 0x7FF) - 1023 - 52
    idx = k >> 6  # floor division (arithmetic shift)
    shift = k - (idx << 6)
    W = _INV2PI

    def word(i):  # Julia's 1-based INV_2PI[i]
        return W[i - 1]
    if shift == 0:
        a1, a2, a3 = word(idx + 1), word(idx + 2), word(idx + 3)
    else:
        a1 = ((0 if idx < 0 else (word(idx + 1) << shift) & M64) | (word(idx + 2) >> (64 - shift)))
        a2 = ((word(idx + 2) << shift) & M64) | (word(idx + 3) >> (64 - shift))
        a3 = ((word(idx + 3) << shift) & M64) | (word(idx + 4) >> (64 - shift))
    w1 = ((X * a1) & M64) << 64
    w2 = X * a2
    w3 = (X * a3) >> 64
    w = (w1 + w2 + w3) & M128  # x/(2π) mod 1, 128-bit fixed point
    if x < 0:
        w = (-w) & M128
    q = ((w >> 125) + 1) >> 1  # nearest quadrant
    f = (w << 2) & M128
    if f >= 1 << 127:
        f -= 1 << 128  # as Int128
    z_hi, z_lo = _fromfraction(f)
    pio2, pio2_hi, pio2_lo = PIO2, PIO2_HI, PIO2_LO
    y_hi = (z_hi + z_lo) * pio2
    y_lo = (((z_hi * pio2_hi - y_hi) + z_hi * pio2_lo) + z_lo * pio2_hi) + z_lo * pio2_lo
    return q, y_hi, y_lo


def rem_pio2(x: float):
    """(n, hi, lo): x = n·π/2 + (hi + lo), |hi + lo| ≲ π/4 (Julia rem_pio2_kernel)."""
    xhp = _poshighword(x)
    if xhp <= 0x400F6A7A:  # |x| ~<= 5π/4
        if (xhp & 0xFFFFF) == 0x921FB:  # |x| ~= π/2 or π
            return _cw_ext(x, xhp)
        if xhp <= 0x4002D97C:  # |x| ~<= 3π/4
            return _cw_2c(x, 1.0, 1) if x > 0.0 else _cw_2c(x, -1.0, -1)
        return _cw_2c(x, 2.0, 2) if x > 0.0 else _cw_2c(x, -2.0, -2)
    if xhp <= 0x401C463B:  # |x| ~<= 9π/4
        if xhp <= 0x4015FDBC:  # |x| ~<= 7π/4
            if xhp == 0x4012D97C:  # |x| ~= 3π/2
                return _cw_ext(x, xhp)
            return _cw_2c(x, 3.0, 3) if x > 0.0 else _cw_2c(x, -3.0, -3)
        if xhp == 0x401921FB:  # |x| ~= 2π
            return _cw_ext(x, xhp)
        return _cw_2c(x, 4.0, 4) if x > 0.0 else _cw_2c(x, -4.0, -4)
    if xhp < 0x413921FB:  # |x| ~< 2^20·π/2
        return _cw_ext(x, xhp)
    return _payne_hanek(x)


SQRT_EPS = math.sqrt(2.0 ** -52)
SQRT_HALF_EPS = math.sqrt(2.0 ** -53)


def sin(x: float) -> float:
    ax = abs(x)
    if ax < PI / 4:
        if ax < SQRT_EPS:
            return x
        return sin_kernel(x)
    if math.isnan(x) or math.isinf(x):
        return math.nan
    n, hi, lo = rem_pio2(x)
    n &= 3
    if n == 0:
        return sin_kernel_dd(hi, lo)
    if n == 1:
        return cos_kernel_dd(hi, lo)
    if n == 2:
        return -sin_kernel_dd(hi, lo)
    return -cos_kernel_dd(hi, lo)


def cos(x: float) -> float:
    ax = abs(x)
    if ax < PI / 4:
        if ax < SQRT_HALF_EPS:
            return 1.0
        return cos_kernel_dd(x, 0.0)
    if math.isnan(x) or math.isinf(x):
        return math.nan
    n, hi, lo = rem_pio2(x)
    n &= 3
    if n == 0:
        return cos_kernel_dd(hi, lo)
    if n == 1:
        return -sin_kernel_dd(hi, lo)
    if n == 2:
        return -cos_kernel_dd(hi, lo)
    return sin_kernel_dd(hi, lo)


def sincos(x: float):
    if abs(x) < PI / 4:
        if x == 0.0:
            return x, 1.0
        return sin_kernel(x), cos_kernel_dd(x, 0.0)
    if math.isnan(x) or math.isinf(x):
        return math.nan, math.nan
    n, hi, lo = rem_pio2(x)
    n &= 3
    si, co = sin_kernel_dd(hi, lo), cos_kernel_dd(hi, lo)
    if n == 0:
        return si, co
    if n == 1:
        return co, -si
    if n == 2:
        return -si, -co
    return -co, si


# ---- atan (s_atan.c) ---------------------------------------------------------------------------
ATANHI = [_f(u) for u in (0x3FDDAC670561BB4F, 0x3FE921FB54442D18, 0x3FEF730BD281F69B,
                          0x3FF921FB54442D18)]
ATANLO = [_f(u) for u in (0x3C7A2B7F222F65E2, 0x3C81A62633145C07, 0x3C7007887AF0CBBD,
                          0x3C91A62633145C07)]
AT = [_f(u) for u in (0x3FD555555555550D, 0xBFC999999998EBC4, 0x3FC24924920083FF,
                      0xBFBC71C6FE231671, 0x3FB745CDC54C206E, 0xBFB3B0F2AF749A6D,
                      0x3FB10D66A0D03D51, 0xBFADDE2D52DEFD9A, 0x3FA97B4B24760DEB,
                      0xBFA2B4442C6A6C2F, 0x3F90AD3AE322DA11)]


def atan(x: float) -> float:
    if math.isnan(x):
        return x
    xu = _poshighword(x)
    neg = math.copysign(1.0, x) < 0
    if xu >= 0x44100000:  # |x| ≥ 2^66
        z = ATANHI[3] + ATANLO[3]
        return -z if neg else z
    if xu < 0x3FDC0000:  # |x| < 0.4375
        if xu < 0x3E400000:  # |x| < 2^-27
            return x
        idn = -1
    else:
        x = abs(x)
        if xu < 0x3FF30000:  # |x| < 1.1875
            if xu < 0x3FE60000:  # 7/16 ≤ |x| < 11/16
                idn = 0
                x = (2.0 * x - 1.0) / (2.0 + x)
            else:  # 11/16 ≤ |x| < 19/16
                idn = 1
                x = (x - 1.0) / (x + 1.0)
        else:
            if xu < 0x40038000:  # |x| < 2.4375
                idn = 2
                x = (x - 1.5) / (1.0 + 1.5 * x)
            else:  # 2.4375 ≤ |x| < 2^66
                idn = 3
                x = -1.0 / x
    z = x * x
    w = z * z
    s1 = z * horner(w, AT[0], AT[2], AT[4], AT[6], AT[8], AT[10])
    s2 = w * horner(w, AT[1], AT[3], AT[5], AT[7], AT[9])
    if idn < 0:
        return x - x * (s1 + s2)
    z = ATANHI[idn] - ((x * (s1 + s2) - ATANLO[idn]) - x)
    return -z if neg else z


PI_LO = _f(0x3CA1A62633145C07)


def atan2(y: float, x: float) -> float:
    """Julia's atan(y, x) (e_atan2.c)."""
    if math.isnan(x) or math.isnan(y):
        return x if math.isnan(x) else y
    if x == 1.0:
        return atan(y)
    m = 2 * (math.copysign(1.0, x) < 0) + (math.copysign(1.0, y) < 0)
    if y == 0.0:
        return y if m in (0, 1) else (PI if m == 2 else -PI)
    if x == 0.0:
        return math.copysign(PI / 2, y)
    if math.isinf(x):
        if math.isinf(y):
            return (PI / 4, -PI / 4, 3 * PI / 4, -3 * PI / 4)[m]
        return (0.0, -0.0, PI, -PI)[m]
    if math.isinf(y):
        return math.copysign(PI / 2, y)
    k = _poshighword(y) - _poshighword(x)
    k = (k - (1 << 32) if k >= 1 << 31 else k) >> 20  # Int32 difference, arithmetic shift
    if k > 60:
        z = PI / 2 + 0.5 * PI_LO
        m &= 1
    elif x < 0 and k < -60:
        z = 0.0
    else:
        z = atan(abs(y / x))
    if m == 0:
        return z
    if m == 1:
        return -z
    if m == 2:
        return PI - (z - PI_LO)
    return (z - PI_LO) - PI


def hypot(x: float, y: float) -> float:
    """Julia's hypot (base/math.jl) with a hardware fma for muladd."""
    if math.isinf(x) or math.isinf(y):
        return math.inf
    ax, ay = abs(x), abs(y)
    if ay > ax:
        ax, ay = ay, ax
    if ay <= ax * SQRT_HALF_EPS:
        return ax
    scale = 2.0 ** -52 * math.sqrt(2.0 ** -1022)
    if ax > math.sqrt(sys.float_info.max / 2):
        ax, ay = ax * scale, ay * scale
        scale = 1.0 / scale
    elif ay < math.sqrt(2.0 ** -1022):
        ax, ay = ax / scale, ay / scale
    else:
        scale = 1.0
    h = math.sqrt(fma(ax, ax, ay * ay))
    h_sq = h * h
    ax_sq = ax * ax
    h -= (fma(-ay, ay, h_sq - ax_sq) + fma(h, h, -h_sq) - fma(ax, ax, -ax_sq)) / (2 * h)
    return h * scale
