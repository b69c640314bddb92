"""Float32 per-sample arithmetic (GPD_FP32, method="fp32"): BASELINE config 5's "fp32 vs fp64"
half.  The reference's own Float32 path cannot run (binit = 0.1 is Float64 while the functor
wants b::T, src/Modulation.jl:403, 318), so this is the build's own experiment:
the exact evaluator with θ, sin, sincos, FC phasor, model, products and residual in Float32 on
phases reduced modulo 2π once per call in Float64, sums and NEWUOA in Float64.  Its reference is
the Float64 exact path (itself the oracle's bits); the tolerance here is the experiment's
measured envelope (tools/c5_sweep.py reports the full sweep), not a parity claim."""
import numpy as np
import pytest

import synth
from test_gpu_parity import faint_states

pytestmark = pytest.mark.gpu


def _dev(x, r):
    dphi = np.abs((x["phi"] - r["phi"] + np.pi) % (2 * np.pi) - np.pi)
    return np.max([np.abs(x["b"] - r["b"]) / np.abs(r["b"]), dphi,
                   np.abs(x["a"] - r["a"]) / np.abs(r["a"])], axis=0)


@pytest.mark.parametrize("faint", [False, True])
def test_fp32_arithmetic_close_to_fp64(gpu, faint):
    N, P = 20_000, 64
    B = synth.make_batch(N, P, seed=11)
    st = None
    if faint:
        st = faint_states(N, seed=4)
        B["d"] = B["d"] * np.where(st == 3, 1.1, np.where(st == 1, 0.01, 0.1))[None, :]
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    ref = gpu.fit_batch(*args, state=st, method="exact")
    got = gpu.fit_batch(*args, state=st, method="fp32")
    assert np.all(got["status"] & gpu.GPD_ST_EXACT)
    assert not np.any(got["status"] & gpu.GPD_ST_NAN)
    e = _dev(got, ref)
    print(f"fp32 vs fp64 exact (faint={faint}): median {np.median(e):.1e}, max {e.max():.1e}, "
          f"within 1e-5 {np.mean(e <= 1e-5):.2f}")
    assert e.max() < 1e-3                 # below NEWUOA's rhoend
    assert np.median(e) < 1e-4            # Float32 rounding, not a different fit
    chi = np.abs(got["chi2"] - ref["chi2"]) / ref["chi2"]
    assert np.median(chi) < 1e-5


def test_fp32_records_are_deterministic_and_shard_invariant(gpu, opts):
    B = synth.make_batch(8000, 48, seed=3)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    one = gpu.fit_batch(*args, method="fp32")
    assert gpu.fit_batch(*args, method="fp32").tobytes() == one.tobytes()
    opts("fake_gpus", 1)
    two = gpu.fit_batch(*args, method="fp32", n_gpus=3)
    assert two.tobytes() == one.tobytes()


def test_fp32_rejects_offsets_and_harmonic(gpu):
    B = synth.make_batch(2000, 4, seed=2)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    with pytest.raises(gpu.GpdError):
        gpu.fit_batch(*args, method="fp32", fitoffsets=True)


@pytest.mark.parametrize("storage", ["c64", "c32"])
@pytest.mark.parametrize("faint", [False, True])
def test_fp32_fast_form_equals_general_form(gpu, opts, storage, faint):
    """The Float32-arithmetic evaluator's FAST form (r6: unconditional loads, the ComplexF32
    series read as 8-B elements, a Float32 model cache) gives the general form's records bit for
    bit (option exact_fast = 0 forces the general form), for both storage types, faint or not,
    at one and at two waves per SIMD."""
    N, P = 12_000, 40
    B = synth.make_batch(N, P, seed=17)
    st = None
    if faint:
        st = faint_states(N, seed=6)
        B["d"] = B["d"] * np.where(st == 3, 1.1, np.where(st == 1, 0.01, 0.1))[None, :]
    d, fc = B["d"], B["fc"]
    if storage == "c32":
        d, fc = d.astype(np.complex64), fc.astype(np.complex64)
    args = (B["t"], d, fc, B["fc_of_pixel"])
    for waves in (1, 2):
        opts("exact_waves", waves)
        opts("exact_fast", 1)
        fast = gpu.fit_batch(*args, state=st, method="fp32")
        opts("exact_fast", 0)
        gen = gpu.fit_batch(*args, state=st, method="fp32")
        assert fast.tobytes() == gen.tobytes(), (storage, faint, waves)
