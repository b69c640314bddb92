"""The shared restatement of Julia Base's Float64 sin / cos / sincos / atan / atan(y, x) / hypot /
rem_pio2 (gppupildemodulation.jl_amd/csrc/gpd_jlmath.h): the functions the reference applies per
sample (src/Modulation.jl:137,388,419-421; src/Faint.jl:95-97) and OptimPackNextGen's NEWUOA per
trial angle.  One source is compiled into the oracle (gcc) and the device (hipcc, gfx950).

CPU: the constants are re-derived from exact integer arithmetic, the functions are checked
against correctly rounded values (decimal, 110 digits) and glibc — msun's kernels are within one
ulp and agree with the correctly rounded value for ~97 % of arguments.  Parity of the
restatement with Julia itself stays UNPINNED (no Julia here).
GPU: the device evaluates every function bit for bit as the oracle does, over argument ranges
that take every reduction branch (two-constant and extended Cody–Waite, Payne–Hanek at
MJD-scale arguments) and the special values."""
import math
import os
import re
import sys
from decimal import Decimal, getcontext, localcontext

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "gppupildemodulation.jl_amd", "csrc", "gpd_jlmath.h")
sys.path.insert(0, os.path.join(ROOT, "oracle", "tools"))
import inv2pi  # noqa: E402


def ulps(a, b):
    """Distance in units in the last place between two float64 arrays (same sign or zero)."""
    ai = np.asarray(a, dtype=np.float64).view(np.int64)
    bi = np.asarray(b, dtype=np.float64).view(np.int64)
    lo = np.int64(-0x8000000000000000)
    ai = np.where(ai < 0, lo - ai, ai)
    bi = np.where(bi < 0, lo - bi, bi)
    return np.abs(ai - bi)


def same_bits(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    return np.all(both_nan | (a.view(np.int64) == b.view(np.int64)))


def test_inv2pi_words_and_hypot_thresholds_are_exact():
    text = open(HDR).read()
    start = text.index("#define JLM_INV2PI_WORDS")
    body = text[start:text.index("#if defined(__HIP__)", start)]
    words = [int(w, 16) for w in re.findall(r"0x([0-9a-f]{16})ull", body)]
    assert words == inv2pi.inv2pi_words()
    th = inv2pi.hypot_thresholds()
    assert th["sqrt(eps/2)"] in text and th["sqrt(floatmax/2)"] in text


def argument_sets(rng, n):
    """Every branch of rem_pio2_kernel: |x| < π/4 (no reduction), ≲ 9π/4 (two constants, n=±1..±4),
    near multiples of π/2 (the extended scheme), < 2^20·π/2 (extended), MJD-scale ω·t ≈ 3.3e10 and
    huge arguments (Payne–Hanek)."""
    mult = np.array([k * math.pi / 2 for k in range(-8, 9) if k])
    near = (np.tile(mult, n // 16 + 1) * (1 + rng.uniform(-1e-9, 1e-9, 16 * (n // 16 + 1))))[:n]
    return {
        "small": rng.uniform(-0.785, 0.785, n),
        "quadrants": rng.uniform(-7.1, 7.1, n),
        "near_k_pi_2": near,
        "medium": rng.uniform(-1.6e6, 1.6e6, n),
        "mjd": rng.uniform(3.2e10, 3.4e10, n),
        "huge": np.sign(rng.uniform(-1, 1, n)) * 10.0 ** rng.uniform(7, 300, n),
        "tiny": np.sign(rng.uniform(-1, 1, n)) * 10.0 ** rng.uniform(-320, -7, n),
    }


@pytest.mark.parametrize("fn", ["sin", "cos"])
def test_sin_cos_against_glibc(oracle, fn):
    rng = np.random.default_rng(3)
    ref = np.vectorize(getattr(math, fn))
    for name, x in argument_sets(rng, 40000).items():
        got = oracle.jl_eval(fn, x)
        u = ulps(got, ref(x))
        assert u.max() <= 1, (fn, name, u.max())
        assert (u == 0).mean() >= 0.95, (fn, name, (u == 0).mean())


def _dec_pi(bits=380):
    return Decimal(inv2pi.pi_fixed(bits)) / (Decimal(2) ** bits)


def _dec_sin_cos(x, pi):
    X = Decimal(x)
    k = (X / (pi / 2)).to_integral_value()
    r = X - k * (pi / 2)
    r2 = r * r
    eps = Decimal(10) ** -105
    s = t = r
    n = 1
    while abs(t) > eps:
        t = -t * r2 / ((2 * n) * (2 * n + 1))
        s += t
        n += 1
    c = t = Decimal(1)
    n = 1
    while abs(t) > eps:
        t = -t * r2 / ((2 * n - 1) * (2 * n))
        c += t
        n += 1
    q = int(k) % 4
    return [(s, c), (c, -s), (-s, -c), (-c, s)][q]


def test_sin_cos_against_correctly_rounded(oracle):
    """msun's sin/cos: within one ulp of the correctly rounded value everywhere, equal to it for
    the large majority of arguments (the reduction is exact up to MJD scale)."""
    getcontext().prec = 110
    pi = _dec_pi()
    rng = np.random.default_rng(5)
    for lo, hi in ((-0.785, 0.785), (-10.0, 10.0), (-2e3, 2e3), (1e5, 1.6e6), (3.2e10, 3.4e10)):
        x = rng.uniform(lo, hi, 600)
        sc = [_dec_sin_cos(v, pi) for v in x]
        cr_s = np.array([float(s) for s, _ in sc])
        cr_c = np.array([float(c) for _, c in sc])
        for got, cr in ((oracle.jl_eval("sin", x), cr_s), (oracle.jl_eval("cos", x), cr_c)):
            u = ulps(got, cr)
            assert u.max() <= 1 and (u == 0).mean() >= 0.93, (lo, hi, u.max(), (u == 0).mean())


def test_sincos_is_sin_and_cos(oracle):
    """Julia's sincos returns the very values of sin and cos (exp(Complex(0, β)) and sin(θ) of
    the model agree)."""
    rng = np.random.default_rng(7)
    sets = list(argument_sets(rng, 20000).values())
    # the device NEWUOA's trial angles (TRSAPP / BIGLAG / BIGDEN take one sincos where the
    # oracle's NEWUOA calls cos and sin, gpd_newuoa.hpp): dang·(i + s), s ∈ [-½, ½], and tiny ones
    dang = 6.283185307179586476925286766559 / 50.0
    sets.append(dang * (np.arange(50)[:, None] + np.linspace(-0.5, 0.5, 2001)[None, :]).ravel())
    tiny = np.ldexp(1.0, np.arange(-1074, 3).astype(np.int64))
    sets.append(np.concatenate([tiny, -tiny, 1.3 * tiny]))
    for x in sets:
        sc = oracle.jl_eval("sincos", x)
        assert same_bits(sc[:, 0], oracle.jl_eval("sin", x))
        assert same_bits(sc[:, 1], oracle.jl_eval("cos", x))


def test_rem_pio2_is_an_exact_reduction(oracle):
    """x = n·π/2 + (hi + lo) far beyond double precision of the remainder (msun's design: the
    Cody–Waite rounds stop once ~2^-70 of |hi| is reached, Payne–Hanek keeps ~2^-100; checked in
    420-digit decimal arithmetic)."""
    getcontext().prec = 420  # |x| up to 1e300
    pi = _dec_pi(1500)
    rng = np.random.default_rng(9)
    for name, x in argument_sets(rng, 300).items():
        x = x[np.abs(x) >= 0.7854]  # the callers reduce only |x| ≥ π/4
        if x.size == 0:
            continue
        r = oracle.jl_eval("rem_pio2", x)
        for xi, (q, hi, lo) in zip(x, r):
            assert abs(hi) <= 0.7854 + 1e-9
            exact = Decimal(xi) - Decimal(int(q)) * (pi / 2)
            # Payne–Hanek returns the quadrant modulo 4: compare the remainder modulo 2π
            exact = exact - ((exact - Decimal(hi)) / (2 * pi)).to_integral_value() * 2 * pi
            err = abs(exact - (Decimal(hi) + Decimal(lo)))
            assert err <= Decimal(2) ** -68 * abs(Decimal(hi)), (name, xi, q, hi, lo, err)


def test_atan_atan2_hypot_against_glibc(oracle):
    rng = np.random.default_rng(11)
    n = 100000
    x = rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))
    y = rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))
    u = ulps(oracle.jl_eval("atan", x), np.vectorize(math.atan)(x))
    assert u.max() <= 1 and (u == 0).mean() >= 0.98
    u = ulps(oracle.jl_eval("atan2", y, x), np.vectorize(math.atan2)(y, x))
    assert u.max() <= 1 and (u == 0).mean() >= 0.8
    # Julia's hypot with hardware fma is correctly rounded, as is glibc's
    assert same_bits(oracle.jl_eval("hypot", x, y), np.vectorize(math.hypot)(x, y))


def test_special_values(oracle):
    inf, nan = math.inf, math.nan
    s = oracle.jl_eval("sin", [0.0, -0.0, inf, -inf, nan, 1e-300])
    assert s[0] == 0 and math.copysign(1, s[1]) == -1 and np.isnan(s[2:5]).all() and s[5] == 1e-300
    c = oracle.jl_eval("cos", [0.0, inf, nan])
    assert c[0] == 1.0 and np.isnan(c[1:]).all()
    # angle(Complex(x, y)) = atan(y, x): the quadrant conventions of src/Modulation.jl:388
    y = np.array([0.0, -0.0, 0.0, -0.0, 1.0, -1.0, inf, inf, -inf, 1.0, 2.0, nan])
    x = np.array([1.0, 1.0, -1.0, -1.0, 0.0, 0.0, inf, -inf, 5.0, -inf, 1.0, 1.0])
    ref = np.array([math.atan2(a, b) for a, b in zip(y, x)])
    got = oracle.jl_eval("atan2", y, x)
    assert same_bits(got[:-1], ref[:-1]) and np.isnan(got[-1])
    h = oracle.jl_eval("hypot", [inf, nan, 3.0, 0.0, 1e-310], [nan, inf, 4.0, 0.0, 1e-310])
    assert h[0] == inf and h[1] == inf and h[2] == 5.0 and h[3] == 0.0
    assert h[4] == math.hypot(1e-310, 1e-310)


def _hypot_args(rng, n):
    """Pairs across every path of hypot: ordinary, swapped, ratio below sqrt(eps/2), both
    scaling ranges (> sqrt(floatmax/2), < sqrt(floatmin)), subnormals, ±0, ±Inf, NaN."""
    x = rng.standard_normal(n) * np.exp(rng.uniform(-745, 709, n))
    y = rng.standard_normal(n) * np.exp(rng.uniform(-745, 709, n))
    x[: n // 4] = rng.standard_normal(n // 4) * 2.0 ** 511 * rng.uniform(0.5, 3, n // 4)
    y[: n // 4] = rng.standard_normal(n // 4) * 2.0 ** 511 * rng.uniform(0.1, 3, n // 4)
    x[n // 4: n // 2] = rng.standard_normal(n // 4) * 2.0 ** -520
    y[n // 4: n // 2] = rng.standard_normal(n // 4) * 2.0 ** -505
    y[n // 2: n // 2 + 1000] = x[n // 2: n // 2 + 1000] * 1e-9
    sp = [0.0, -0.0, math.inf, -math.inf, math.nan, 5e-324, -5e-324, 1e-310, 1.0, 2.0 ** 1023,
          float.fromhex("0x1.6a09e667f3bccp+511"), float.fromhex("0x1.6a09e667f3bcdp+511"),
          2.0 ** -511, 2.0 ** -512]
    a, b = np.meshgrid(sp, sp)
    return np.concatenate([x, a.ravel()]), np.concatenate([y, b.ravel()])


def test_branch_free_hypot_equals_hypot(oracle):
    """jl_hypot_nb (every path evaluated, result selected — the faint statistics' hypot) gives
    jl_hypot's bits on every input."""
    x, y = _hypot_args(np.random.default_rng(17), 400000)
    assert same_bits(oracle.jl_eval("hypot_nb", x, y), oracle.jl_eval("hypot", x, y))


@pytest.mark.gpu
def test_device_libm_equals_oracle_bitwise(gpu, oracle):
    """The exact evaluator's per-sample functions on the device = the oracle's, bit for bit."""
    rng = np.random.default_rng(13)
    sets = argument_sets(rng, 50000)
    specials = np.array([0.0, -0.0, math.inf, -math.inf, math.nan, 5e-324, -5e-324, 1e-310,
                         math.pi / 2, math.pi, 3 * math.pi / 2, 2 * math.pi, 1e300, -1e300,
                         2.0 ** 1023, 86400.0 * 60000.0 * 6.283185])
    sets["specials"] = specials
    for name, x in sets.items():
        for fn in ("sin", "cos", "sincos", "atan", "rem_pio2"):
            if fn == "rem_pio2":
                x = x[np.isfinite(x) & (np.abs(x) >= 0.7854)]
            d, h = gpu.libm_eval(fn, x), oracle.jl_eval(fn, x)
            assert same_bits(d, h), (fn, name, np.nonzero(~(d.view(np.int64) == h.view(np.int64)))[0][:5])
    n = 200000
    xs = rng.standard_normal(n) * np.exp(rng.uniform(-40, 40, n))
    ys = rng.standard_normal(n) * np.exp(rng.uniform(-40, 40, n))
    xs[:16] = specials
    ys[:16] = specials[::-1]
    for fn in ("atan2", "hypot", "hypot_nb"):
        assert same_bits(gpu.libm_eval(fn, xs, ys), oracle.jl_eval(fn, xs, ys)), fn
    hx, hy = _hypot_args(rng, 200000)
    assert same_bits(gpu.libm_eval("hypot_nb", hx, hy), oracle.jl_eval("hypot", hx, hy))


def _trig_regime_args(rng, n):
    """Arguments of every regime the branch-free forms cover and of their edges: MJD-scale ωt
    (Payne–Hanek, shift 0 exponents included), Cody–Waite extended, |β| ≲ 9π/4 with the
    extended-precision points π/2, π, 3π/2, 2π and their neighbours, ±0, tiny, inf, NaN."""
    k = np.arange(1, 9) * (np.pi / 2)
    near = np.concatenate([np.nextafter(k, np.inf), np.nextafter(k, -np.inf), k,
                           k * (1 + 1e-7), k * (1 - 1e-7)])
    edges = np.array([2.0 ** 20 * np.pi / 2, np.nextafter(2.0 ** 20 * np.pi / 2, 0), 9 * np.pi / 4,
                      np.nextafter(9 * np.pi / 4, 0), np.nextafter(9 * np.pi / 4, 10), np.pi / 4,
                      np.nextafter(np.pi / 4, 0), 0.0, -0.0, 5e-324, 1e-300, 2.0 ** -27,
                      np.inf, -np.inf, np.nan, 2.0 ** 1023, 1.7e308])
    shift0 = np.ldexp(1.0 + rng.random(2000), rng.integers(1, 16, 2000) * 64 + 11)  # k ≡ 0 mod 64
    # Payne–Hanek arguments close to multiples of π/2 (small fractions: short normalisations in
    # fromfraction), and the classic hardest case of double-precision reduction
    k2 = np.ldexp(np.pi / 2, np.arange(21, 1000))
    close = np.concatenate([k2, np.nextafter(k2, np.inf), np.nextafter(k2, 0),
                            [6381956970095103.0 * 2.0 ** 797]])
    sets = [rng.uniform(3.2e10, 3.5e10, n) + rng.uniform(-np.pi, np.pi, n),  # MJD·ω + ϕ
            np.exp(rng.uniform(np.log(7.0), np.log(1.6e6), n)) * rng.choice([-1, 1], n),
            rng.uniform(-7.2, 7.2, n), rng.uniform(-2.6, 2.6, n),
            np.exp(rng.uniform(np.log(1.7e6), 700, n // 4)), shift0, close, -close, near, -near,
            edges, -edges]
    return np.concatenate(sets)


def test_branch_free_sin_sincos_equal_the_general_functions(oracle):
    """jl_sin_ph_nb / jl_sin_cwx_nb / jl_sincos_small_nb (every branch of the regime evaluated,
    the exact evaluator's batched model) give jl_sin's and jl_sincos's bits inside their regimes;
    outside them the dispatch falls back to the general functions."""
    x = _trig_regime_args(np.random.default_rng(29), 300000)
    assert same_bits(oracle.jl_eval("sin_sel", x), oracle.jl_eval("sin", x))
    assert same_bits(oracle.jl_eval("sincos_sel", x), oracle.jl_eval("sincos", x))


@pytest.mark.gpu
def test_device_branch_free_trig_equals_oracle(gpu, oracle):
    """The device's branch-free regime forms (the exact evaluator's batched model) = jl_sin and
    jl_sincos of the oracle, bit for bit, on every regime and edge."""
    x = _trig_regime_args(np.random.default_rng(31), 200000)
    assert same_bits(gpu.libm_eval("sin_sel", x), oracle.jl_eval("sin", x))
    assert same_bits(gpu.libm_eval("sincos_sel", x), oracle.jl_eval("sincos", x))


PI60 = "3.14159265358979323846264338327950288419716939937510582097494"


def _ph_shift_cases(rng):
    """(x array in one binade, ϕ) pairs: MJD-scale exposures at 500 Hz, ϕ over ±8 rad, θ = x + ϕ
    next to multiples of π/2 (Payne–Hanek's cancellation cases), the binade's edges, ϕ at exact
    half-ulp ties and at integer ulps, ±0."""
    cases = []
    for _ in range(120):
        t0 = 86400.0 * rng.uniform(50000, 62000)
        t = t0 + np.arange(int(rng.integers(2, 2500))) * 0.002
        x = 6.283185 * t
        for phi in list(rng.uniform(-8, 8, 4)) + [0.0, -0.0, math.pi, -math.pi / 2]:
            cases.append((x, phi))
    # θ within a few ulps of n·π/2 (leading zeros of Payne–Hanek's fraction)
    for k in range(200):
        e = int(rng.integers(25, 40))
        n = int(rng.integers(2 ** (e - 1), 2 ** e)) * 4 + int(rng.integers(0, 4))
        with localcontext() as ctx:  # the double nearest n·π/2, π to 60 digits
            ctx.prec = 80
            th = float(Decimal(n) * Decimal(PI60) / 2)
        phi = float(rng.uniform(-3, 3))
        x = np.nextafter(th - phi, np.inf * (k % 2 - 0.5)) + np.zeros(3)
        x[1] = np.nextafter(x[0], np.inf)
        x[2] = np.nextafter(x[0], -np.inf)
        cases.append((x, phi))
    # the binade's edges, and ϕ exactly on ties / whole ulps of the binade
    for e in (25, 34, 35, 41):
        lo, hi = 2.0 ** e, 2.0 ** (e + 1)
        u = 2.0 ** (e - 52)
        for base in (lo, hi - 64 * u, lo + 1e3 * u):
            x = base + np.arange(64) * u
            for phi in (0.5 * u, -0.5 * u, 7.5 * u, 3 * u, -3 * u, 70 * u, -70 * u, 0.3 * u):
                cases.append((x, phi))
    return cases


def test_payne_hanek_shift_equals_payne_hanek(oracle):
    """jl_sin(fl(x + ϕ)) from the per-sample Payne–Hanek table of x and the per-evaluation shift
    of ϕ (gpd_jlmath.h jlm_ph_table_entry / jlm_ph_shift / jl_sin_ph_shifted, r6: the exact
    evaluator's MJD path): wherever the shift applies, the bits of jl_sin of the rounded sum; it
    declines (NaN) exactly where θ's mantissa is not X + rint(ϕ/u) for every x — ties of ϕ/u, a θ
    that could leave the binade — and everywhere it declines the evaluator takes the general form."""
    rng = np.random.default_rng(61)
    n_on = n_all = 0
    for x, phi in _ph_shift_cases(rng):
        got = oracle.jl_eval("sin_ph_shift", x, np.full(x.size, phi))
        ref = oracle.jl_eval("sin", x + phi)
        on = ~np.isnan(got)
        assert same_bits(got[on], ref[on]).all(), (x[:3], phi)
        e = np.frexp(x)[1]
        u = np.ldexp(1.0, int(e[0]) - 53)
        r = phi / u
        tie = abs(r - np.rint(r)) == 0.5
        one_binade = (e == e[0]).all() and (np.frexp(x + phi)[1] == e[0]).all()
        if on.any():
            assert not tie and one_binade
        elif one_binade and not tie and x.min() > 2 ** 21 and abs(r) < 2 ** 40:
            # declined only at the binade's edges (X + rint(r) ± 1 outside it)
            X = np.frexp(x)[0] * 2.0 ** 53
            assert (X.min() + np.rint(r) - 1 < 2 ** 52) or (X.max() + np.rint(r) + 1 > 2 ** 53 - 1)
        n_on += int(on.sum())
        n_all += x.size
    assert n_on > 0.9 * n_all, (n_on, n_all)


@pytest.mark.gpu
def test_device_payne_hanek_shift_equals_oracle(gpu, oracle):
    """The device's Payne–Hanek table entry and shifted sin (k_libm fn 10, the code the exact
    evaluator's first pass runs on MJD-scale phases) give the oracle's bits, and so jl_sin's of
    the rounded sum, on the same cases as the CPU test."""
    rng = np.random.default_rng(62)
    n = 0
    for x, phi in _ph_shift_cases(rng)[::3]:
        y = np.full(x.size, phi)
        got = gpu.libm_eval("sin_ph_shift", x, y)
        ref = oracle.jl_eval("sin_ph_shift", x, y)
        on = ~np.isnan(ref)
        assert (np.isnan(got) == ~on).all() and same_bits(got[on], ref[on]).all(), (x[:2], phi)
        n += int((~np.isnan(got)).sum())
    assert n > 0
