"""CPU checks of the oracle (test infrastructure) against known answers and the reference's
stated properties.  PARITY UNPINNED: the reference ships no tests/fixtures and cannot run here,
so these pin the restatement with (a) bit-exact Julia constants, (b) published NEWUOA behaviour
on standard problems, (c) mathematical identities of the model, (d) truth recovery."""
import json
import math
import os
import sys

import numpy as np
import pytest

import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_phi_grid_is_julia_range(oracle):
    sys.path.insert(0, os.path.join(ROOT, "oracle", "tools"))
    import phi_grid

    ref = phi_grid.julia_range(-math.pi, math.pi, 8)
    np.testing.assert_array_equal(oracle.phi_grid(), np.array(ref))
    assert oracle.phi_grid()[0] == -math.pi and oracle.phi_grid()[-1] == math.pi


def test_newuoa_rosenbrock(oracle):
    f = lambda x: (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2
    x, fx, nf = oracle.newuoa(f, [-1.2, 1.0], 0.5, 1e-8, maxfun=2000)
    np.testing.assert_allclose(x, [1.0, 1.0], atol=1e-6)
    assert fx < 1e-12 and nf < 400


def test_newuoa_quadratic_exact_minimum(oracle):
    f = lambda x: (x[0] - 3) ** 2 + 2 * (x[1] + 1) ** 2 + x[0] * x[1]
    x, fx, nf = oracle.newuoa(f, [0.0, 0.0], 1.0, 1e-7, maxfun=500)
    np.testing.assert_allclose(x, [4.0, -2.0], atol=1e-6)
    assert abs(fx + 5.0) < 1e-12


def test_newuoa_respects_maxfun(oracle):
    f = lambda x: (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2
    _, _, nf = oracle.newuoa(f, [-1.2, 1.0], 0.5, 1e-8, maxfun=60)
    assert nf == 60


def _series(seed=4, N=4000, offsets=False):
    B = synth.make_batch(N, 4, seed=seed, offsets=offsets)
    p = np.exp(1j * np.angle(B["fc"][0]))
    return B, p


def test_chi2_symmetry_b_phi(oracle):
    """f(b, ϕ) = f(−b, ϕ + π) (tex/GPPupilDemodulation.tex:189)."""
    B, p = _series()
    for b, phi in [(0.7, 0.3), (1.9, -2.0), (2.6, 3.0)]:
        f1, _ = oracle.chi2(B["t"], B["d"][0], p, b, phi)
        f2, _ = oracle.chi2(B["t"], B["d"][0], p, -b, phi + math.pi)
        assert abs(f1 - f2) <= 1e-12 * f1


@pytest.mark.parametrize("offsets", [False, True])
def test_chi2_closed_form_is_least_squares(oracle, offsets):
    """a (and c) from the closed form (src/Modulation.jl:140-146) are the LS solution; χ² is the
    weighted residual norm / N (src/Modulation.jl:320)."""
    B, p = _series(offsets=offsets)
    t, d = B["t"], B["d"][0]
    b, phi = 1.3, 0.4
    f, rec = oracle.chi2(t, d, p, b, phi, offsets=offsets)
    m = p * np.exp(1j * b * np.sin(6.283185 * t + phi))
    A = np.stack([np.ones_like(m), m], 1) if offsets else m[:, None]
    sol, *_ = np.linalg.lstsq(A, d, rcond=None)
    if offsets:
        np.testing.assert_allclose([rec["c"], rec["a"]], sol, rtol=1e-10, atol=1e-12)
    else:
        np.testing.assert_allclose(rec["a"], sol[0], rtol=1e-12)
    r = A @ sol - d
    assert abs(f - np.sum(np.abs(r) ** 2) / len(d)) <= 1e-12 * f


def test_fit_recovers_truth(oracle):
    B = synth.make_batch(20000, 16, seed=11)
    par = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    tr = B["truth"]
    # noise-limited: σ=0.1 complex noise, 2e4 samples → parameter errors ~1e-3
    assert np.max(np.abs(par["b"] - tr["b"])) < 1e-2
    assert np.max(synth.wrap(par["phi"] - tr["phi"]).__abs__()) < 1e-2
    assert np.max(np.abs(np.abs(par["a"]) - np.abs(tr["a"]))) < 1e-2
    assert np.all(np.abs(par["chi2"] - 0.01) < 1e-3)  # E|noise|² = σ²
    assert np.all(par["b"] >= 0)  # sign normalisation


@pytest.mark.parametrize("order", [1, 16, 32])
def test_alternative_summation_orders(oracle, order):
    """The reference-ceiling probe (bench.py): the cost's sums in another order a CPU may take
    (sequential, or a vectorised loop with 16 / 32 accumulators).  χ² at a fixed point moves by
    ulps only; the fits stay the same minimum to NEWUOA's rhoend; order 0 is CR8 itself."""
    B = synth.make_batch(4000, 8, seed=9)
    a = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    ref = oracle.fit_batch(*a, flags=oracle.RECENTER)
    same = oracle.fit_batch(*a, flags=oracle.RECENTER, order=0)
    assert np.array_equal(same, ref)
    alt = oracle.fit_batch(*a, flags=oracle.RECENTER, order=order)
    assert np.all(np.abs(alt["b"] - ref["b"]) <= 1e-3 * np.abs(ref["b"]))
    assert np.all(np.abs(alt["chi2"] - ref["chi2"]) <= 1e-6 * ref["chi2"])
    # the order really differs: the fitted χ² bits are not all equal
    assert not np.array_equal(alt["chi2"], ref["chi2"])
    with pytest.raises(ValueError):
        oracle.fit_batch(*a, order=7)


def test_mean_var_power_matches_numpy(oracle):
    rng = np.random.default_rng(0)
    d = rng.standard_normal(3000) + 1j * rng.standard_normal(3000)
    st = rng.choice(np.array([0, 1, 2, 3], dtype=np.int8), size=3000)
    m, w = oracle.mean_var_power(st, d)
    for s in range(4):
        sel = st == s
        a = np.abs(d[sel])
        np.testing.assert_allclose(m[sel], a.mean(), rtol=1e-13)
        np.testing.assert_allclose(w[sel], 1 / a.var(ddof=1), rtol=1e-12)


@pytest.mark.parametrize("level,noise", [(1.0, 0.3), (1.0, 1e-2), (1e3, 1e-3), (1e-6, 1e-9)])
@pytest.mark.parametrize("onlyhigh", [False, True])
def test_fused_mean_var_power_matches_two_pass(oracle, level, noise, onlyhigh):
    """The fused one-pass statistics (shifted sums, K = abs(d) at each state's first valid
    sample; the device's state-split moment pass, r4) against the two-pass restatement of
    compute_mean_var_power (src/Faint.jl:89-100): m within 1e-15, w within 1e-13 relative — the
    stated tolerance — also at |d|/σ ≈ 1e3, where the raw one-pass form Σx² − (Σx)²/n loses
    six digits (and misses the tolerance by 1e3×)."""
    rng = np.random.default_rng(int(level * 1e6) % 1000 + int(onlyhigh))
    N = 20_000
    st = rng.choice(np.array([0, 1, 2, 3, -1], dtype=np.int8), size=N, p=[0.1, 0.3, 0.3, 0.25, 0.05])
    amp = np.where(st == 3, 1.1, np.where(st == 1, 0.3, 0.6)) * level
    ph = rng.uniform(-np.pi, np.pi, N)
    d = (amp + noise * level * rng.standard_normal(N)) * np.exp(1j * ph)
    m2, w2 = oracle.mean_var_power_series(st, d, onlyhigh=onlyhigh)
    m1, w1 = oracle.mean_var_power_fused(st, d, onlyhigh=onlyhigh)
    ok = np.isfinite(w2)
    assert ok[1:].sum() >= (2 if onlyhigh else 4)
    np.testing.assert_allclose(m1[ok], m2[ok], rtol=1e-15)
    np.testing.assert_allclose(w1[ok], w2[ok], rtol=1e-13)
    assert np.isnan(m1[0]) and np.isnan(w1[0])  # TRANSIENT: never valid
    if level == 1e3:  # the raw one-pass form the shift avoids
        valid = (st == 3) & ~(np.isnan(d))
        a = np.abs(d[valid])
        raw = (np.sum(a * a) - np.sum(a) ** 2 / a.size) / (a.size - 1)
        assert abs(1 / raw / w2[4] - 1) > 1e-11


def test_mean_var_power_single_sample_state_is_nan(oracle):
    d = np.ones(10, dtype=np.complex128) * (1 + 1j)
    st = np.full(10, 2, dtype=np.int8)
    st[3] = 0
    m, w = oracle.mean_var_power(st, d)
    assert np.isnan(w[3]) and np.isfinite(w[0])


def py_buildstates(t, t1, t2, pre, post, s1=3, s2=1):
    """Line-by-line Python transcription of src/Faint.jl:21-73 (lag = 0)."""
    step = t[1] - t[0]
    premax, postmax = math.ceil(pre / step), math.ceil(post / step)
    t1, t2 = list(t1), list(t2)
    cur, f1, f2, forget, out = 2, t1.pop(0), t2.pop(0), 0, []
    for time in t:
        if time >= f1:
            cur, forget = s1, premax
            if not t1:
                f1 = t[-1]
                if f2 == t[-1]:
                    cur = 2
            else:
                f1 = t1.pop(0)
        if time >= f2:
            cur, forget = s2, postmax
            if not t2:
                f2 = t[-1]
                if f1 == t[-1]:
                    cur = 2
            else:
                f2 = t2.pop(0)
        if forget > 0:
            out.append(-1)
            forget -= 1
        else:
            out.append(cur)
    return np.array(out, dtype=np.int8)


@pytest.mark.parametrize("pre,post", [(0.0, 0.0), (0.01, 0.3), (0.004, 0.02)])
def test_buildstates(oracle, pre, post):
    t = np.arange(3000) * 0.002 + 1.0
    t1 = 1.0 + np.arange(5) * 1.1 + 0.3    # HIGH switches
    t2 = t1 + 0.35                          # LOW switches
    got = oracle.buildstates(t, t1, t2, preswitchdelay=pre, postwitchdelay=post)
    np.testing.assert_array_equal(got, py_buildstates(t, t1, t2, pre, post))
    assert set(np.unique(got)) <= {-1, 1, 2, 3}


def test_golden_fixtures_reproduce(oracle):
    """Regression fixtures (tests/golden/, generated by tests/golden/make_golden.py from the
    oracle on seeded synthetic inputs).  Pins the oracle against silent changes."""
    path = os.path.join(ROOT, "tests", "golden", "oracle_fits.json")
    golden = json.load(open(path))
    for case in golden["cases"]:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        import make_golden

        got = make_golden.run_case(oracle, case["spec"])
        for key in ("b", "phi", "chi2", "a_re", "a_im"):
            np.testing.assert_allclose(got[key], case["expect"][key], rtol=1e-12, atol=1e-14,
                                       err_msg=f"{case['spec']['name']}:{key}")
        np.testing.assert_array_equal(got["nfev"], case["expect"]["nfev"])


def event_buildstates(t, t1, t2, pre, post):
    """The firing-list formulation of gpd_states.hpp (k_bs_prep / k_bs_events / k_bs_fill) in
    Python: checks the reduction itself against the line-by-line transcription on CPU."""
    n, n1, n2 = t.size, len(t1), len(t2)
    step = t[1] - t[0]
    premax, postmax = math.ceil(pre / step), math.ceil(post / step)
    tl = t[-1]
    lb = np.searchsorted(t, np.concatenate([t1, t2]), side="left")
    lbT = int(np.searchsorted(t, tl, side="left"))
    last = np.concatenate([t1, t2]) == tl
    c1 = c2 = 0
    l1 = l2 = -1
    cur = 2
    ev = []
    while True:
        k1 = max(l1 + 1, lb[c1] if c1 < n1 else lbT)
        k2 = max(l2 + 1, lb[n1 + c2] if c2 < n2 else lbT)
        k1, k2 = (k1 if k1 < n else n), (k2 if k2 < n else n)
        k = min(k1, k2)
        if k >= n:
            break
        fg = 0
        if k1 == k:
            cur, fg = 3, premax
            if c1 >= n1 - 1:
                c1 = n1
                if c2 >= n2 or last[n1 + c2]:
                    cur = 2
            else:
                c1 += 1
            l1 = k
        if k2 == k:
            cur, fg = 1, postmax
            if c2 >= n2 - 1:
                c2 = n2
                if c1 >= n1 or last[c1]:
                    cur = 2
            else:
                c2 += 1
            l2 = k
        ev.append((k, cur, fg))
    out = np.full(n, 2, dtype=np.int8)
    ks = np.array([e[0] for e in ev], dtype=np.int64)
    for k in range(n):
        j = np.searchsorted(ks, k, side="right") - 1
        if j >= 0:
            ek, es, ef = ev[j]
            out[k] = -1 if k - ek < ef else es
    return out


def random_timer_case(rng):
    """Edge cases of src/Faint.jl:21-73: entries closer than Δt (the one-pop-per-sample lag),
    before t[0], after and exactly at t[N-1], repeated final timestamps, single entries."""
    n = int(rng.integers(2, 400))
    t = 10.0 + np.arange(n) * 0.002
    if rng.random() < 0.3:
        t[-int(rng.integers(1, 4)):] = t[-1] if n > 4 else t[-1]
        t = np.maximum.accumulate(t)
    span = t[-1] - t[0]

    def timer():
        m = int(rng.integers(1, 8))
        x = t[0] + rng.uniform(-0.1, 1.1, m) * span
        if rng.random() < 0.3:
            x = np.concatenate([x, x[:1] + rng.uniform(0, 0.003, 2)])  # within one interval
        if rng.random() < 0.2:
            x[rng.integers(0, x.size)] = t[-1]
        return np.sort(x)

    pre, post = (0.0, 0.0) if rng.random() < 0.3 else (rng.uniform(0, 0.05), rng.uniform(0, 0.2))
    return t, timer(), timer(), pre, post


def test_event_formulation_equals_reference_loop():
    rng = np.random.default_rng(5)
    for _ in range(400):
        t, t1, t2, pre, post = random_timer_case(rng)
        np.testing.assert_array_equal(event_buildstates(t, t1, t2, pre, post),
                                      py_buildstates(t, t1, t2, pre, post))
