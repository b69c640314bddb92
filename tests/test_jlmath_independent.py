"""The shared Julia-Base libm restatement (gpd_jlmath.h, compiled into the oracle and the device)
against a second, independent restatement written in Python from the same published algorithms
(oracle/tools/jlmath_py.py: Julia's base/special/trig.jl, rem_pio2.jl and base/math.jl over
FreeBSD msun), bit for bit, on arguments that take every branch: the small-argument kernels and
their cut-offs, two-constant and extended Cody–Waite reduction (including the points next to
π/2, π, 3π/2, 2π that switch to the extended scheme), the medium Payne–Hanek reduction up to
1e300 and at MJD-scale phases, atan's five intervals and atan(y, x)'s special cases, hypot's
scaling ranges.  A transcription slip in the header that stays within an ulp of glibc — which
the accuracy tests of tests/test_jlmath.py cannot see — fails here unless both transcriptions
make it.  Julia itself is absent, so parity with Julia stays unpinned."""
import math
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle", "tools"))
import jlmath_py as jp  # noqa: E402


def _trig_args(rng, n):
    pio2 = math.pi / 2
    parts = [
        rng.uniform(-math.pi / 4, math.pi / 4, n),
        np.exp(rng.uniform(math.log(1e-12), math.log(1.0), n)) * rng.choice([-1, 1], n),
        rng.uniform(-10.0, 10.0, n),  # two-constant reduction, n = ±1..±4
        np.exp(rng.uniform(math.log(10.0), math.log(1.6e6), n)) * rng.choice([-1, 1], n),  # extended
        np.exp(rng.uniform(math.log(1.7e6), math.log(1e22), n)) * rng.choice([-1, 1], n),  # Payne–Hanek
        np.exp(rng.uniform(math.log(1e22), math.log(1e300), n // 4)),
        # MJD-scale phases fl(ωt), t ≈ 86400·MJD (the reference's absolute timestamps)
        2 * math.pi * (86400.0 * 60000.0 + rng.uniform(0, 3600.0, n)),
        # next to multiples of π/2 (extended-scheme switch points and large k)
        np.concatenate([k * pio2 + rng.uniform(-1e-6, 1e-6, n // 8) for k in (1, 2, 3, 4, -1, -2, -3, -4)]),
        rng.integers(1, 1 << 20, n) * pio2 + rng.uniform(-1e-9, 1e-9, n),
    ]
    edges = []
    for hw in (0x3E500000, 0x3E46A09E, 0x3FE921FB, 0x4002D97C, 0x400F6A7A, 0x4012D97C,
               0x4015FDBC, 0x401921FB, 0x401C463B, 0x413921FB):
        for lw in (0, 1, 0x54442D18, 0xFFFFFFFF):
            edges.append(jp._f((hw << 32) | lw))
    edges += [math.pi / 4, np.nextafter(math.pi / 4, 0), np.nextafter(math.pi / 4, 4), 0.0, -0.0,
              5e-324, 2.2250738585072014e-308, 1.4901161193847656e-08]
    a = np.concatenate(parts + [np.array(edges), -np.array(edges)])
    return a[np.isfinite(a)]


def _check(name, got, want, args):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    bad = ~(((got.view(np.int64)) == want.view(np.int64)) | (np.isnan(got) & np.isnan(want)))
    if bad.any():
        i = np.flatnonzero(bad)[:5]
        raise AssertionError(f"{name}: {bad.sum()} of {bad.size} differ, e.g. "
                             + "; ".join(f"{args[j]!r}: header {got[j]!r} vs python {want[j]!r}"
                                         for j in i))


def test_sin_cos_sincos_rem_pio2_match_the_independent_restatement(oracle):
    rng = np.random.default_rng(20251017)
    x = _trig_args(rng, 1500)
    for fn, ref in (("sin", jp.sin), ("cos", jp.cos)):
        _check(fn, oracle.jl_eval(fn, x), [ref(float(v)) for v in x], x)
    sc = oracle.jl_eval("sincos", x)
    want = np.array([jp.sincos(float(v)) for v in x])
    _check("sincos.sin", sc[:, 0], want[:, 0], x)
    _check("sincos.cos", sc[:, 1], want[:, 1], x)
    big = x[np.abs(x) >= math.pi / 4]
    rp = oracle.jl_eval("rem_pio2", big)
    want = np.array([jp.rem_pio2(float(v)) for v in big], dtype=object)
    n_ok = np.array([int(rp[i, 0]) % 4 == int(want[i, 0]) % 4 for i in range(big.size)])
    assert n_ok.all(), f"rem_pio2 quadrant differs at {big[~n_ok][:5]}"
    _check("rem_pio2.hi", rp[:, 1], want[:, 1].astype(np.float64), big)
    _check("rem_pio2.lo", rp[:, 2], want[:, 2].astype(np.float64), big)


def test_atan_atan2_match_the_independent_restatement(oracle):
    rng = np.random.default_rng(7)
    n = 3000
    mags = np.exp(rng.uniform(math.log(1e-30), math.log(1e30), n))
    edges = [0.4375, 0.6875, 1.1875, 2.4375, 2.0 ** 66, 2.0 ** -27, 1.0, 0.0, -0.0, math.inf]
    edges += [np.nextafter(e, 0) for e in edges[:6]] + [np.nextafter(e, 10 * e) for e in edges[:6]]
    x = np.concatenate([mags * rng.choice([-1, 1], n), rng.uniform(-3, 3, n), edges,
                        -np.array(edges)])
    _check("atan", oracle.jl_eval("atan", x), [jp.atan(float(v)) for v in x], x)
    # atan(y, x): jl_eval("atan2", y, x)
    yy = np.exp(rng.uniform(math.log(1e-300), math.log(1e300), n)) * rng.choice([-1, 1], n)
    xx = np.exp(rng.uniform(math.log(1e-300), math.log(1e300), n)) * rng.choice([-1, 1], n)
    near = rng.uniform(-2, 2, (2, n))
    specials = [0.0, -0.0, 1.0, -1.0, math.inf, -math.inf, 1e-310, 3.0]
    sy, sx = np.meshgrid(specials, specials)
    Y = np.concatenate([yy, near[0], sy.ravel(), xx[:50] * 2.0 ** 61])
    X = np.concatenate([xx, near[1], sx.ravel(), xx[:50]])
    _check("atan2", oracle.jl_eval("atan2", Y, X), [jp.atan2(float(a), float(b)) for a, b in zip(Y, X)],
           list(zip(Y, X)))


def test_hypot_matches_the_independent_restatement(oracle):
    rng = np.random.default_rng(11)
    n = 4000
    a = np.exp(rng.uniform(math.log(1e-310), math.log(1e288), n)) * rng.choice([-1, 1], n)
    b = a * np.exp(rng.uniform(math.log(1e-20), math.log(1e20), n)) * rng.choice([-1, 1], n)
    c = rng.normal(size=(2, n))
    specials = [0.0, -0.0, 1.0, math.inf, -math.inf, 5e-324, 1e300, 1.3407807929942596e154]
    sx, sy = np.meshgrid(specials, specials)
    X = np.concatenate([a, c[0], sx.ravel()])
    Y = np.concatenate([b, c[1], sy.ravel()])
    want = [jp.hypot(float(u), float(v)) for u, v in zip(X, Y)]
    _check("hypot", oracle.jl_eval("hypot", X, Y), want, list(zip(X, Y)))
    _check("hypot_nb", oracle.jl_eval("hypot_nb", X, Y), want, list(zip(X, Y)))


@pytest.mark.parametrize("fn", ["sin", "cos"])
def test_independent_restatement_is_within_an_ulp_of_glibc(fn):
    """The Python restatement is itself a faithful libm (so the agreement above is between two
    accurate transcriptions, not two copies of one error)."""
    rng = np.random.default_rng(3)
    x = _trig_args(rng, 200)
    ref = getattr(math, fn)
    got = np.array([getattr(jp, fn)(float(v)) for v in x])
    want = np.array([ref(float(v)) for v in x])
    d = np.abs(got.view(np.int64) - want.view(np.int64))
    assert np.all(d <= 1), x[d > 1][:5]
