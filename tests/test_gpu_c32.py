"""Float32-storage entry points (gpd_fit_batch_c32 / gpd_fit_windows_c32; BASELINE config 5).

The series and FC columns stay ComplexF32 in HBM (the FITS VOLT precision) and are widened to
Float64 as they are loaded, so the fit sees exactly Float64.(data).  Parity therefore has two
parts: (1) the c32 path is BIT-IDENTICAL to the Float64 path run on the widened arrays (same
kernels' arithmetic on the same values — every evaluator, faint and windowed paths included);
(2) the oracle on the widened arrays, with the same tie-envelope criterion as every fit test.
"""
import numpy as np
import pytest

import synth
from test_gpu_parity import (assert_fit_parity, faint_batch, oracle_fit, perturbed_runs,
                             ulps_for)

pytestmark = pytest.mark.gpu

FIELDS = ("c", "a", "b", "phi", "chi2", "nfev", "status")


def c32_batch(N, P, seed, faint=False):
    if faint:
        B, st = faint_batch(N, P, seed)
    else:
        B, st = synth.make_batch(N, P, seed=seed), None
    B32 = dict(B, d=B["d"].astype(np.complex64), fc=B["fc"].astype(np.complex64))
    B64 = dict(B, d=B32["d"].astype(np.complex128), fc=B32["fc"].astype(np.complex128))
    return B32, B64, st


def assert_identical(a, b, label):
    for f in FIELDS:
        x, y = a[f], b[f]
        same = (x == y) | ((x != x) & (y != y))
        assert np.all(same), f"{label}: field {f} differs at {np.nonzero(~same)[0][:5]}"


@pytest.mark.parametrize("faint", [False, True])
@pytest.mark.parametrize("method", ["exact", "harmonic"])
def test_c32_equals_widened_f64(gpu, method, faint):
    B32, B64, st = c32_batch(5000, 40, seed=31, faint=faint)
    args = lambda B: (B["t"], B["d"], B["fc"], B["fc_of_pixel"])  # noqa: E731
    got, out32 = gpu.fit_batch(*args(B32), state=st, method=method, want_output=True)
    ref, out64 = gpu.fit_batch(*args(B64), state=st, method=method, want_output=True)
    assert_identical(got, ref, f"c32/{method}/faint={faint}")
    assert np.array_equal(out32, out64)


def test_c32_offsets_and_ragged(gpu):
    """fitoffsets (exact and harmonic G-moment path over Float32 FC columns), ragged P."""
    B32, B64, _ = c32_batch(4099, 133, seed=32)
    B32["d"] = B32["d"] + np.complex64(0.05 - 0.03j)
    B64["d"] = B32["d"].astype(np.complex128)
    for method in ("exact", "harmonic"):
        got = gpu.fit_batch(B32["t"], B32["d"], B32["fc"], B32["fc_of_pixel"], fitoffsets=True,
                            method=method)
        ref = gpu.fit_batch(B64["t"], B64["d"], B64["fc"], B64["fc_of_pixel"], fitoffsets=True,
                            method=method)
        assert_identical(got, ref, f"c32 offsets/{method}")


@pytest.mark.parametrize("faint", [False, True])
def test_c32_windows_equal_widened(gpu, faint):
    B32, B64, st = c32_batch(9000, 32, seed=33, faint=faint)
    fop = B32["fc_of_pixel"]
    got = gpu.fit_windows(B32["t"], B32["d"], B32["fc"], fop, 1500, state=st)
    ref = gpu.fit_windows(B64["t"], B64["d"], B64["fc"], fop, 1500, state=st)
    for w in range(got.shape[0]):
        assert_identical(got[w], ref[w], f"c32 windows w={w}")


def test_c32_matches_oracle(gpu, oracle):
    """Oracle on the widened data (the values the reference would see after Float64.(VOLT))."""
    B32, B64, _ = c32_batch(6000, 48, seed=34)
    got = gpu.fit_batch(B32["t"], B32["d"], B32["fc"], B32["fc_of_pixel"])
    ref = oracle_fit(oracle, B64)
    pert = perturbed_runs(oracle, B64, ulps=ulps_for("harmonic"))
    print(assert_fit_parity(got, ref, pert, label="c32/auto"))


def test_demodulateall_keeps_complex64(gpu):
    """demodulateall on a Matrix{ComplexF32}: output = copy(data) keeps the element type
    (src/Modulation.jl:353); fits equal those of the widened matrix."""
    B32, B64, _ = c32_batch(3000, 32, seed=35)
    t = B32["t"]
    data32 = np.empty((t.size, 40), dtype=np.complex64)
    data32[:, :32] = B32["d"].T
    data32[:, 32:] = B32["fc"].T
    out32, par32, lk32 = gpu.demodulateall(t, data32)
    out64, par64, lk64 = gpu.demodulateall(t, data32.astype(np.complex128))
    assert out32.dtype == np.complex64
    assert np.array_equal(lk32, lk64)
    assert all(p.b == q.b and p.ϕ == q.ϕ and p.a == q.a for p, q in zip(par32, par64))
    assert np.array_equal(out32, out64.astype(np.complex64))
