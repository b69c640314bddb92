"""Faint power and weight on the GPU (§8 row a10): compute_mean_var_power (src/Faint.jl:89-100)
as demodulateall applies it (valid mask, src/Modulation.jl:373-396) — the one-pass kernels
(k_faint_p1/p2/fin: one hypot per sample, |d| through a MALL-sized scratch, cohorts of series)
and the two-pass kernel (GPD_FAINT_STATS=2; the windows' kernel) against the oracle, bit for bit,
NaN for empty / 1-sample states included."""
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
def test_mean_var_power_matches_oracle(gpu, oracle, monkeypatch, kernel, onlyhigh, N):
    if kernel == "two-pass":
        monkeypatch.setenv("GPD_FAINT_STATS", "2")
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
def test_one_pass_equals_two_pass(gpu, monkeypatch, N, P):
    """The two kernels give the same bits on every length (a part with no sample, ragged last
    slots) and across several cohorts (300 series × 1e5 samples = 2 cohorts of ≤ 239)."""
    d, st = _series(N, P, seed=3)
    a = gpu.mean_var_power_batch(st, d)
    monkeypatch.setenv("GPD_FAINT_STATS", "2")
    b = gpu.mean_var_power_batch(st, d)
    assert _bits(a[0], b[0]) and _bits(a[1], b[1])


@pytest.mark.parametrize("method", ["exact", "harmonic"])
def test_faint_fit_same_with_either_kernel(gpu, monkeypatch, method):
    d, st = _series(30_000, 16, seed=9)
    B = synth.make_batch(30_000, 16, seed=9)
    args = (B["t"], d, B["fc"], B["fc_of_pixel"])
    st = np.where(st == 0, 2, st).astype(np.int8)  # no 1-sample state: finite fits
    a = gpu.fit_batch(*args, state=st, method=method)
    monkeypatch.setenv("GPD_FAINT_STATS", "2")
    b = gpu.fit_batch(*args, state=st, method=method)
    assert a.tobytes() == b.tobytes()
