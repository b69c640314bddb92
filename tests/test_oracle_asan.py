"""The oracle under AddressSanitizer + UndefinedBehaviorSanitizer (verdict r5 item 8).

`make -C oracle asan` compiles the oracle's sources — NEWUOA, the cost and driver, the faint
statistics, buildstates and the product's shared Julia-Base libm restatement (gpd_jlmath.h) —
with -fsanitize=address,undefined -fno-sanitize-recover=all behind a command-line driver
(oracle/asan_driver.c).  These tests feed it the inputs of the oracle's own test cases (edge
lengths, faint states with empty and one-sample states, NaNs, fitoffsets, xinit, the buildstates
edge cases, every libm regime) and require (1) a clean exit with no sanitizer report and (2) the
same results as the ordinary liboracle.so, bit for bit.  CPU only.
"""
import fcntl
import os
import struct
import subprocess

import numpy as np
import pytest

import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "oracle", "_asan", "asan_driver")


@pytest.fixture(scope="module")
def asan():
    # one build at a time (pytest-xdist workers would otherwise relink the driver while another
    # worker runs it)
    os.makedirs(os.path.dirname(DRIVER), exist_ok=True)
    with open(DRIVER + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"],
                           capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(DRIVER)

    def run(payload: bytes) -> bytes:
        env = dict(os.environ, OMP_NUM_THREADS="4",
                   ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
        r = subprocess.run([DRIVER], input=payload, capture_output=True, env=env, timeout=600)
        err = r.stderr.decode(errors="replace")
        assert r.returncode == 0 and "Sanitizer" not in err and "runtime error" not in err, \
            f"sanitizer build failed (rc {r.returncode}):\n{err[-4000:]}"
        return r.stdout
    return run


def _fit_job(t, d, fc, fop, state=None, xinit=None, flags=2, maxfun=60, want_out=False,
             nthreads=4, seed=0, ulps=1.0, omega=synth.M_2PI):
    N = t.size
    P = d.shape[0]
    b = struct.pack("<iqqqIiiiiiQdd", 1, N, P, fc.shape[0], flags, maxfun, nthreads,
                    state is not None, xinit is not None, want_out, seed, omega, ulps)
    b += np.ascontiguousarray(t, np.float64).tobytes()
    b += np.ascontiguousarray(d, np.complex128).tobytes()
    b += np.ascontiguousarray(fc, np.complex128).tobytes()
    b += np.ascontiguousarray(fop, np.int32).tobytes()
    if state is not None:
        b += np.ascontiguousarray(state, np.int8).tobytes()
    if xinit is not None:
        b += np.ascontiguousarray(xinit, np.float64).tobytes()
    return b


def _read_fit(out, P, N, want_out):
    rc = struct.unpack_from("<i", out)[0]
    assert rc == 0
    o = 4
    import oracle as O
    par = np.frombuffer(out, dtype=O.PARAM_DTYPE, count=P, offset=o).copy()
    o += 64 * P
    dem = None
    if want_out:
        dem = np.frombuffer(out, dtype=np.complex128, count=P * N, offset=o).reshape(P, N).copy()
        o += 16 * P * N
    return par, dem, out[o:]


def _same_records(a, b):
    for k in ("b", "phi", "chi2"):
        x, y = a[k], b[k]
        assert np.all((x == y) | (np.isnan(x) & np.isnan(y))), k
    for k in ("a", "c"):
        for part in ("real", "imag"):
            x, y = getattr(a[k], part), getattr(b[k], part)
            assert np.all((x == y) | (np.isnan(x) & np.isnan(y))), k
    np.testing.assert_array_equal(a["nfev"], b["nfev"])
    np.testing.assert_array_equal(a["status"], b["status"])


def _faint_states(N, seed):
    rng = np.random.default_rng(seed)
    st = np.full(N, 2, dtype=np.int8)
    i = N // 10
    while i < N - N // 10:
        hi = int(rng.integers(max(1, N // 40), max(2, N // 20)))
        st[i:i + hi] = 3
        st[i:i + 5] = -1
        lo = int(rng.integers(max(1, N // 20), max(2, N // 8)))
        st[i + hi:i + hi + lo] = 1
        st[i + hi:i + hi + 15] = -1
        i += hi + lo
    return st


FIT_CASES = [
    # (N, P, kwargs) — tile / block / chain edges of the canonical order, tiny series
    dict(N=2, P=2),
    dict(N=37, P=3),
    dict(N=2049, P=4),
    dict(N=4000, P=8, want_out=True),
    dict(N=4000, P=8, flags=3, want_out=True),                 # fitoffsets
    dict(N=3000, P=4, flags=0, xinit=np.array([0.7, -0.4])),   # recenter off, xinit
    dict(N=3000, P=4, faint=True),
    dict(N=3000, P=4, faint=True, flags=6),                    # onlyhigh
    dict(N=3000, P=4, seed=3, ulps=128.0),                     # the perturbed runs
    dict(N=2500, P=4, nan=True),                               # NaN samples → status NAN
    dict(N=600, P=4, maxfun=7),                                # maxfun reached
]


@pytest.mark.parametrize("case", FIT_CASES, ids=lambda c: "-".join(f"{k}{v if not isinstance(v, np.ndarray) else ''}" for k, v in c.items()))
def test_fit_batch_under_sanitizers(asan, oracle, case):
    c = dict(case)
    N, P = c.pop("N"), c.pop("P")
    B = synth.make_batch(N, P, seed=5 + N % 7, offsets=bool(c.get("flags", 2) & 1))
    state = _faint_states(N, N) if c.pop("faint", False) else None
    if state is not None and N >= 3000:
        state[:3] = 0   # OFF samples: a state with no weight
        state[-1] = 1
    d = B["d"].copy()
    if c.pop("nan", False):
        d[1, N // 3] = np.nan
    want = c.get("want_out", False)
    out = asan(_fit_job(B["t"], d, B["fc"], B["fc_of_pixel"], state=state, **c))
    par, dem, rest = _read_fit(out, P, N, want)
    assert rest == b""
    ref = oracle.fit_batch(B["t"], d, B["fc"], B["fc_of_pixel"], state=state,
                           xinit=c.get("xinit"), flags=c.get("flags", 2),
                           maxfun=c.get("maxfun", 60), want_output=want,
                           perturb_seed=c.get("seed", 0), perturb_ulps=c.get("ulps", 1.0))
    if want:
        ref, refout = ref
        np.testing.assert_array_equal(dem, refout)
    _same_records(par, ref)


def test_chi2_and_statistics_under_sanitizers(asan, oracle):
    N = 5000
    B = synth.make_batch(N, 2, seed=11, offsets=True)
    st = _faint_states(N, 4)
    st[100] = 0  # a one-sample state: w = NaN as Julia's 0/0
    p = oracle.fc_phasor(B["fc"][0])
    w = np.random.default_rng(1).uniform(0.5, 2.0, N)
    payload = b""
    pts = [(0.3, 1.2, 0, None), (2.4, -2.9, 1, None), (1.1, 0.4, 0, w), (3.7, 3.0, 1, w)]
    for b, phi, offs, ww in pts:
        payload += struct.pack("<iqiiddd", 2, N, offs, ww is not None, synth.M_2PI, b, phi)
        payload += B["t"].tobytes() + B["d"][0].tobytes() + p.tobytes()
        if ww is not None:
            payload += ww.tobytes()
    for flags in (0, 4):
        for fused in (0, 1):
            payload += struct.pack("<iqIi", 4, N, flags, fused) + st.tobytes() + B["d"][1].tobytes()
    out = asan(payload)
    o = 0
    import oracle as O
    for b, phi, offs, ww in pts:
        v = struct.unpack_from("<d", out, o)[0]
        rec = np.frombuffer(out, dtype=O.PARAM_DTYPE, count=1, offset=o + 8)[0]
        o += 8 + 64
        rv, rrec = oracle.chi2(B["t"], B["d"][0], p, b, phi, w=ww, offsets=bool(offs))
        assert v == rv and rec["a"] == rrec["a"] and rec["c"] == rrec["c"]
    for flags in (0, 4):
        for fused in (0, 1):
            m5 = np.frombuffer(out, np.float64, 5, o)
            w5 = np.frombuffer(out, np.float64, 5, o + 40)
            o += 80
            fn = oracle.mean_var_power_fused if fused else oracle.mean_var_power_series
            rm, rw = fn(st, B["d"][1], onlyhigh=bool(flags))
            np.testing.assert_array_equal(m5, rm)
            np.testing.assert_array_equal(w5, rw)
    assert o == len(out)


def test_buildstates_under_sanitizers(asan, oracle):
    """The buildstates edge cases of tests/test_oracle.py's random sweep (timers before, inside
    and after the exposure, equal times, exhausted lists, zero delays) plus the argument errors."""
    rng = np.random.default_rng(9)
    cases = []
    for k in range(120):
        n = int(rng.integers(2, 400))
        t = np.cumsum(rng.uniform(0.5, 1.5, n)) * 0.002 + rng.uniform(-1, 1)
        n1, n2 = int(rng.integers(1, 12)), int(rng.integers(1, 12))
        lo, hi = t[0] - 0.1, t[-1] + 0.1
        t1 = np.sort(rng.uniform(lo, hi, n1))
        t2 = np.sort(rng.uniform(lo, hi, n2))
        if k % 7 == 0:
            t2[:] = t1[0]  # equal times
        pre, post = (0.0, 0.0) if k % 5 == 0 else (rng.uniform(0, 0.05), rng.uniform(0, 0.3))
        cases.append((t, t1, t2, pre, post))
    cases.append((np.array([0.0]), np.array([0.0]), np.array([1.0]), 0.0, 0.0))  # n < 2: error
    payload = b""
    for t, t1, t2, pre, post in cases:
        payload += struct.pack("<iqqqbbdd", 3, t.size, t1.size, t2.size, 3, 1, pre, post)
        payload += t.tobytes() + t1.tobytes() + t2.tobytes()
    out = asan(payload)
    o = 0
    for t, t1, t2, pre, post in cases:
        rc = struct.unpack_from("<i", out, o)[0]
        got = np.frombuffer(out, np.int8, t.size, o + 4)
        o += 4 + t.size
        if rc != 0:
            with pytest.raises(ValueError):
                oracle.buildstates(t, t1, t2, 3, 1, pre, post)
            continue
        np.testing.assert_array_equal(got, oracle.buildstates(t, t1, t2, 3, 1, pre, post))
    assert o == len(out)


def test_libm_and_newuoa_under_sanitizers(asan, oracle):
    """Every regime of the shared libm restatement (small arguments, Cody–Waite, Payne–Hanek up
    to 1e300 and at MJD-scale phases, atan's intervals, hypot's scalings, NaN/Inf) and NEWUOA on
    the chained Rosenbrock function."""
    rng = np.random.default_rng(2)
    x = np.concatenate([
        rng.uniform(-1e-8, 1e-8, 200), rng.uniform(-10, 10, 400), rng.uniform(-1e5, 1e5, 200),
        3.3e10 + rng.uniform(-1e3, 1e3, 200), 10.0 ** rng.uniform(5, 300, 200),
        np.pi / 2 * np.arange(1, 9), [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 1.7e308]])
    y = np.concatenate([rng.normal(size=x.size - 7) * 10.0 ** rng.uniform(-300, 300, x.size - 7),
                        [0.0, 1.0, np.inf, np.nan, -0.0, 1e-310, -1e308]])
    fns = [(name, code) for name, code in oracle.JL_FN.items()]
    payload = b""
    for name, code in fns:
        two = name in ("atan2", "hypot", "hypot_nb", "sin_ph_shift")
        payload += struct.pack("<iiiq", 5, code, int(two), x.size) + x.tobytes()
        if two:
            payload += y.tobytes()
    starts = [(2, 5, 60, 1.0, 1e-3, [0.1, 0.3]), (2, 5, 400, 0.5, 1e-6, [-1.2, 1.0]),
              (4, 9, 800, 0.5, 1e-6, [-1.2, 1.0, -1.2, 1.0]), (3, 7, 40, 1.0, 1e-3, [0, 0, 0])]
    for n, npt, mf, rb, re_, x0 in starts:
        payload += struct.pack("<iiiidd", 6, n, npt, mf, rb, re_) + np.array(x0, float).tobytes()
    out = asan(payload)
    o = 0
    for name, code in fns:
        two = name in ("atan2", "hypot", "hypot_nb", "sin_ph_shift")
        width = {2: 2, 6: 3, 9: 2}.get(code, 1)
        rc = struct.unpack_from("<i", out, o)[0]
        got = np.frombuffer(out, np.float64, x.size * width, o + 4)
        o += 4 + 8 * x.size * width
        assert rc == 0, name
        ref = oracle.jl_eval(name, x, y if two else None).ravel()
        assert np.array_equal(got, ref, equal_nan=True), name

    def rosen(v):
        f = 0.0
        for i in range(v.size - 1):
            a, b = v[i + 1] - v[i] * v[i], 1.0 - v[i]
            f += 100.0 * a * a + b * b
        return f
    for n, npt, mf, rb, re_, x0 in starts:
        nf = struct.unpack_from("<i", out, o)[0]
        xs = np.frombuffer(out, np.float64, n, o + 4)
        fx = struct.unpack_from("<d", out, o + 4 + 8 * n)[0]
        o += 4 + 8 * n + 8
        rx, rfx, rnf = oracle.newuoa(rosen, np.array(x0, float), rb, re_, maxfun=mf, npt=npt)
        assert nf == rnf and np.array_equal(xs, rx) and fx == rfx
    assert o == len(out)
