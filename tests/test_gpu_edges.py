"""GPU edge cases: ragged shapes (N not a multiple of the 32-sample tile, P not a multiple of
the 128-series workgroup or of 4), a general fc_of_pixel (series not grouped by FC column —
the per-series FC path of both moment kernels), FC samples equal to 0 (angle(0) = 0), NaN
samples, and the smallest series."""
import numpy as np
import pytest

import synth
from test_gpu_parity import assert_exact_bitwise, assert_fit_parity, perturbed_runs, ulps_for

pytestmark = pytest.mark.gpu


def run_both(gpu, oracle, B, label, methods=("exact", "harmonic"), **kw):
    ref = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], flags=oracle.RECENTER)
    for method in methods:
        got = gpu.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], method=method, **kw)
        if method == "exact":
            print(assert_exact_bitwise(got, ref, label=f"{label}/exact"))
            continue
        print(assert_fit_parity(got, ref, perturbed_runs(oracle, B, ulps=ulps_for(method)),
                                label=f"{label}/{method}"))


@pytest.mark.parametrize("N,P", [(1037, 7), (4099, 133), (3000, 258)])
def test_ragged_shapes(gpu, oracle, N, P):
    run_both(gpu, oracle, synth.make_batch(N, P, seed=N + P), f"ragged {N}x{P}")


def test_general_fc_assignment(gpu, oracle):
    """fc_of_pixel not grouped by 4: every workgroup takes the per-series FC path."""
    B = synth.make_batch(3000, 40, seed=8)
    rng = np.random.default_rng(1)
    perm = rng.permutation(40)
    B["d"] = B["d"][perm]
    B["fc_of_pixel"] = np.ascontiguousarray(B["fc_of_pixel"][perm])
    run_both(gpu, oracle, B, "general fc")


def test_fc_zero_samples_take_angle_zero(gpu, oracle):
    B = synth.make_batch(2500, 16, seed=12)
    B["fc"][:, 100:140] = 0.0  # angle(0) = 0 → phasor 1 (src/Modulation.jl:388)
    run_both(gpu, oracle, B, "fc zeros")


def test_nan_sample_propagates(gpu, oracle):
    B = synth.make_batch(2000, 8, seed=14)
    B["d"][3, 500] = np.nan
    for method in ("exact", "harmonic"):
        got = gpu.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], method=method)
        ref = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"])
        assert np.isnan(ref["chi2"][3]) and np.isnan(got["chi2"][3])
        assert got["status"][3] & gpu.GPD_ST_NAN
        ok = np.arange(8) != 3
        assert np.all(np.isfinite(got["chi2"][ok]))


@pytest.mark.parametrize("kernel", [None, "valu"])
def test_nan_fc_sample_propagates(gpu, oracle, opts, kernel):
    """A NaN in a fibre-coupler column: exp(im·angle(NaN)) is NaN (src/Modulation.jl:388), so
    every diode sharing that column ends with a NaN χ² and status NAN — for both evaluators and
    both harmonic moment kernels; the exact evaluator gives the oracle's records bit for bit."""
    if kernel:
        opts("moments", {"valu": 1}[kernel])
    B = synth.make_batch(2000, 12, seed=15)
    g = 1
    B["fc"][g, 700] = complex(np.nan, 0.0)
    hit = B["fc_of_pixel"] == g
    assert hit.sum() == 4
    ref = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], flags=oracle.RECENTER)
    assert np.all(np.isnan(ref["chi2"][hit])) and np.all(np.isfinite(ref["chi2"][~hit]))
    for method in ("exact", "harmonic"):
        got = gpu.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], method=method)
        assert np.all(np.isnan(got["chi2"][hit])), (method, got["chi2"][hit])
        assert np.all(got["status"][hit] & gpu.GPD_ST_NAN)
        assert np.all(np.isfinite(got["chi2"][~hit]))
        assert not np.any(got["status"][~hit] & gpu.GPD_ST_NAN)
        if method == "exact":
            print(assert_exact_bitwise(got, ref, label="nan fc/exact"))


def test_quantised_phase_margin_sends_far_phi_to_exact(gpu, oracle):
    """MJD-scale timestamps (harmonic mode 1: ϕ quantised to the ulp of fl(ωt)): an evaluation at
    |ϕ| beyond the binade margin 2π + 2 is not trusted — the series is re-fitted by the exact
    evaluator (status FALLBACK), which gives the oracle's record bit for bit."""
    B = synth.make_batch(3000, 8, seed=16, t0=86400.0 * 60000.0)
    xinit = np.array([0.8, 9.5])  # starts outside the margin
    ref = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], flags=oracle.RECENTER,
                           xinit=xinit)
    got = gpu.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], xinit=xinit, method="auto")
    assert np.all(got["status"] & gpu.GPD_ST_FALLBACK)
    print(assert_exact_bitwise(got, ref, label="phi margin fallback"))
    bphi = np.stack([np.full(8, 0.8), np.linspace(-9.0, 9.0, 8)], 1)
    h = gpu.chi2_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], bphi, method="harmonic")
    far = np.abs(bphi[:, 1]) > 2 * np.pi + 2
    assert np.all((h["status"][far] & gpu.GPD_ST_FALLBACK) != 0)
    assert not np.any(h["status"][~far] & gpu.GPD_ST_FALLBACK)


def test_two_samples(gpu, oracle):
    """The smallest series the API accepts (n_samples = 2): the χ² minimum is a degenerate flat
    valley, where NEWUOA's landing point follows every ulp of χ² — the exact evaluator computes
    the oracle's bits, so it lands where the oracle does."""
    B = synth.make_batch(2, 4, seed=2)
    ref = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    got = gpu.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], method="exact")
    print(assert_exact_bitwise(got, ref, label="N=2"))


@pytest.mark.parametrize("kernel", ["valu", "ws_f64"])
@pytest.mark.parametrize("faint", [False, True])
def test_alternative_moment_kernels(gpu, oracle, opts, kernel, faint):
    """The VALU kernel (used when a series row or the cos/sin table exceeds the producer/consumer
    kernel's 32-bit buffer offsets) gives the same fits, and so does the producer/consumer kernel
    with every harmonic on the f64 MFMAs (option mix = 0)."""
    from test_gpu_parity import faint_states
    N, P = 3000, 40
    B = synth.make_batch(N, P, seed=77)
    st = None
    flags = oracle.RECENTER
    if faint:
        st = faint_states(N, seed=5)
        B["d"] = B["d"] * np.where(st == 3, 1.1, np.where(st == 1, 0.3, 0.6))[None, :]
    if kernel == "ws_f64":
        opts("mix", 0)
    else:
        opts("moments", {"valu": 1}[kernel])
    got = gpu.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], state=st, method="harmonic")
    ref = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], state=st, flags=flags)
    pert = [oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], state=st, flags=flags,
                             perturb_seed=s, perturb_ulps=128.0) for s in range(1, 13)]
    print(assert_fit_parity(got, ref, pert, label=f"{kernel}/faint={faint}"))


def test_release_and_reuse(gpu, oracle):
    """Host-buffer calls reuse a cached device arena; gpd_release frees it (and the fit
    workspace) and the next call re-allocates: identical results across the three calls."""
    B = synth.make_batch(3000, 16, seed=12)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    a = gpu.fit_batch(*args, want_output=True)
    b = gpu.fit_batch(*args, want_output=True)
    assert gpu.load().gpd_release(0) == 0
    assert gpu.load().gpd_release(999) == gpu._lib.GPD_E_ARG
    c = gpu.fit_batch(*args, want_output=True)
    for x in (b, c):
        np.testing.assert_array_equal(x[0], a[0])
        np.testing.assert_array_equal(x[1], a[1])


def test_c_host_example_runs(gpu, tmp_path):
    """examples/demod_exposure.c: one exposure (32 diodes + 8 FC columns) through gpd_fit_batch
    from plain C recovers every diode's b."""
    import subprocess
    from test_abi import _build_c_example
    exe = _build_c_example(tmp_path / "demod_exposure")
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-1000:]
    assert "ok: 32/32" in r.stdout


@pytest.mark.parametrize("N", [5, 20, 33, 95])
def test_short_series_harmonic_chi2(gpu, N):
    """Series shorter than one 32-sample tile (and one tile + a few samples): the moment kernel's
    padded table tile (bf16 fragments in rows 0..15, zero rows past N) and the partial-tile masking
    give the χ² of the exact evaluator."""
    B = synth.make_batch(N, 12, seed=N)
    rng = np.random.default_rng(N)
    bphi = np.stack([rng.uniform(-3, 3, 12), rng.uniform(-4, 4, 12)], 1)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"], bphi)
    h = gpu.chi2_batch(*args, method="harmonic")
    e = gpu.chi2_batch(*args, method="exact")
    assert not (h["status"] & 0x18).any()
    np.testing.assert_allclose(h["chi2"], e["chi2"], rtol=1e-12, atol=0)
