"""Faint power and weight on the GPU (§8 rows a10, f2): compute_mean_var_power (src/Faint.jl:89-100)
as demodulateall applies it (valid mask, src/Modulation.jl:373-396).
- The separate kernels (the exact evaluator's statistics and gpd_mean_var_power): one-pass
  k_faint_p1/p2/fin (one hypot per sample, |d| through a scratch) and the two-pass kernel
  (option faint_stats = 2; the windows' kernel) against the oracle, bit for bit, NaN for empty /
  1-sample states included.
- The fused statistics of the whole-exposure harmonic path (r4: formed by the state-split moment
  pass's producer waves, k_faint_fused_fin; one HBM pass for faint series) against the two-pass
  oracle within the stated tolerance: m 1e-14, w 1e-13 relative (shifted sums; |q| = |p̄ d|
  instead of hypot(d), the device's tile order instead of the canonical one)."""
import numpy as np
import pytest

import synth
from test_gpu_parity import faint_states

pytestmark = pytest.mark.gpu


def _bits(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return np.all((a == b) | (np.isnan(a) & np.isnan(b)))


def _series(N, P, seed):
    B = synth.make_batch(N, P, seed=seed)
    st = faint_states(N, seed=seed)
    st[N // 3] = 0  # a single OFF sample: var of one sample → NaN weight (src/Faint.jl:97)
    power = np.where(st == 3, 1.1, np.where(st == 1, 0.3, 0.6))
    return B["d"] * power[None, :], st


@pytest.mark.parametrize("kernel", ["one-pass", "two-pass"])
@pytest.mark.parametrize("onlyhigh", [False, True])
@pytest.mark.parametrize("N", [6000, 100_000])
def test_mean_var_power_matches_oracle(gpu, oracle, opts, kernel, onlyhigh, N):
    if kernel == "two-pass":
        opts("faint_stats", 2)
    d, st = _series(N, 12, seed=N % 97)
    m5, w5 = gpu.mean_var_power_batch(st, d, onlyhigh=onlyhigh)
    for k in range(d.shape[0]):
        rm, rw = oracle.mean_var_power_series(st, d[k], onlyhigh=onlyhigh)
        assert _bits(m5[k], rm), (k, m5[k], rm)
        assert _bits(w5[k], rw), (k, w5[k], rw)
    if not onlyhigh:
        assert np.isnan(w5[:, 1]).all()  # OFF: one sample
    assert np.isfinite(m5[:, 4]).all() and np.isfinite(w5[:, 4]).all()  # HIGH


def test_compute_mean_var_power_is_the_reference_function(gpu, oracle):
    """The Python mirror of compute_mean_var_power(states, data): per-sample (m, w) vectors."""
    d, st = _series(20_000, 1, seed=5)
    st = np.where(st == -1, 2, st).astype(np.int8)  # no TRANSIENT: the function has no mask
    m, w = gpu.compute_mean_var_power(st, d[0])
    rm, rw = oracle.mean_var_power(st, d[0])
    assert _bits(m, rm) and _bits(w, rw)


@pytest.mark.parametrize("N,P", [(2047, 8), (131_073, 8), (100_000, 300)])
def test_one_pass_equals_two_pass(gpu, opts, N, P):
    """The two kernels give the same bits on every length (a part with no sample, ragged last
    slots) and across several cohorts (300 series × 1e5 samples = 2 cohorts of ≤ 239)."""
    d, st = _series(N, P, seed=3)
    a = gpu.mean_var_power_batch(st, d)
    opts("faint_stats", 2)
    b = gpu.mean_var_power_batch(st, d)
    assert _bits(a[0], b[0]) and _bits(a[1], b[1])


@pytest.mark.parametrize("method", ["exact", "harmonic"])
def test_faint_fit_same_with_either_kernel(gpu, opts, method):
    """The separate kernels (one-pass, two-pass) give the same fits bit for bit (the harmonic
    path takes them with option faint_stats = 1|2 instead of its fused statistics)."""
    d, st = _series(30_000, 16, seed=9)
    B = synth.make_batch(30_000, 16, seed=9)
    args = (B["t"], d, B["fc"], B["fc_of_pixel"])
    st = np.where(st == 0, 2, st).astype(np.int8)  # no 1-sample state: finite fits
    opts("faint_stats", 1)
    a = gpu.fit_batch(*args, state=st, method=method)
    opts("faint_stats", 2)
    b = gpu.fit_batch(*args, state=st, method=method)
    assert a.tobytes() == b.tobytes()


def _check_fused(m, w, st, d, oracle, onlyhigh):
    worst_m = worst_w = 0.0
    for k in range(d.shape[0]):
        rm, rw = oracle.mean_var_power_series(st, d[k], onlyhigh=onlyhigh)
        for q in range(1, 5):
            if not np.isfinite(rm[q]):  # no sample of this state
                assert np.isnan(m[k, q]) and np.isnan(w[k, q]), (k, q)
                continue
            em = abs(m[k, q] / rm[q] - 1)
            assert em <= 1e-14, (k, q, m[k, q], rm[q])
            worst_m = max(worst_m, em)
            if np.isnan(rw[q]):  # one sample: var = 0/0
                assert np.isnan(w[k, q]), (k, q, w[k, q])
                continue
            ew = abs(w[k, q] / rw[q] - 1)
            assert ew <= 1e-13, (k, q, w[k, q], rw[q])
            worst_w = max(worst_w, ew)
    return worst_m, worst_w


@pytest.mark.parametrize("N,P,onlyhigh,c32", [(6000, 40, False, False), (100_000, 140, False, False),
                                              (100_000, 64, True, False), (30_000, 36, False, True),
                                              (2047, 8, False, False)])
def test_fused_statistics_match_oracle(gpu, oracle, opts, N, P, onlyhigh, c32):
    """The harmonic whole-exposure fit's faint statistics come from its moment pass (fused,
    r4): every series' m and w against the two-pass oracle within 1e-14 / 1e-13 relative,
    NaN where the oracle has no sample / one sample; the χ² aggregates Σw|d|², Σw m² n,
    Σ(w m)²|d|² against the separate kernels' within 1e-13."""
    d, st = _series(N, P, seed=N % 89 + P)
    B = synth.make_batch(N, P, seed=N % 89 + P)
    fc = B["fc"]
    if c32:
        d, fc = d.astype(np.complex64), fc.astype(np.complex64)
    args = (B["t"], d, fc, B["fc_of_pixel"])
    gpu.fit_batch(*args, state=st, onlyhigh=onlyhigh, method="harmonic")
    m, w, agg = gpu.last_faint_stats(P)
    dw = d.astype(np.complex128)
    wm, ww = _check_fused(m, w, st, dw, oracle, onlyhigh)
    print(f"fused statistics N={N} P={P}: max rel m {wm:.2e}, w {ww:.2e}")
    opts("faint_stats", 1)
    gpu.fit_batch(*args, state=st, onlyhigh=onlyhigh, method="harmonic")
    m1, w1, agg1 = gpu.last_faint_stats(P)
    np.testing.assert_allclose(agg, agg1, rtol=1e-13)


def test_fused_statistics_deferred_samples(gpu, oracle):
    """Valid states changing inside 32-sample tiles (runs of 1..40 samples, no TRANSIENT margin):
    the samples whose state differs from their tile's go through k_moments_fix, whose sums
    join the fused statistics — still within the tolerance of the two-pass oracle."""
    N, P = 12_000, 24
    rng = np.random.default_rng(8)
    st = np.empty(N, np.int8)
    i = 0
    while i < N:
        n = int(rng.integers(1, 41))
        st[i:i + n] = rng.choice([1, 2, 3, 0], p=[0.3, 0.3, 0.3, 0.1])
        i += n
    st[rng.integers(0, N, 60)] = -1
    B = synth.make_batch(N, P, seed=29)
    power = np.where(st == 3, 1.1, np.where(st == 1, 0.3, 0.6))
    d = B["d"] * power[None, :]
    gpu.fit_batch(B["t"], d, B["fc"], B["fc_of_pixel"], state=st, method="harmonic")
    m, w, _ = gpu.last_faint_stats(P)
    _check_fused(m, w, st, d, oracle, False)
