"""GPU parity of the windowed batch (processmetrology `window`, src/GPPupilDemodulation.jl:191-225):
every window of every diode against the oracle run on that window's slice — exactly what the
reference does, one demodulateall(times[I], cmplxV[I,:]; state[I]) per window (:204-205)."""
import numpy as np
import pytest

import synth
from test_gpu_parity import assert_exact_bitwise, assert_fit_parity, faint_states, ulps_for

NPERTURB = 24  # short windows: more outcomes per series to sample

pytestmark = pytest.mark.gpu


def exposure(N, seed):
    B = synth.make_batch(N, 32, seed=seed)
    return B


def oracle_windows(oracle, B, nwindow, fop_rows, state=None, flags=None, ulps=1.0, **kw):
    """Oracle per window; returns params (n_windows, C) and perturbed runs of the same shape."""
    N = B["t"].size
    flags = oracle.RECENTER if flags is None else flags
    ref, pert = [], [[] for _ in range(NPERTURB)]
    for s0 in range(0, N, nwindow):
        I = slice(s0, min(N, s0 + nwindow))
        st = None if state is None else state[I]
        args = (B["t"][I], B["d"][:, I], B["fc"][:, I], fop_rows)
        ref.append(oracle.fit_batch(*args, state=st, flags=flags, **kw))
        for j in range(NPERTURB):
            pert[j].append(oracle.fit_batch(*args, state=st, flags=flags, perturb_seed=j + 1,
                                            perturb_ulps=ulps, **kw))
    return np.stack(ref), [np.stack(p) for p in pert]


@pytest.mark.parametrize("method", ["auto", "exact"])
@pytest.mark.parametrize("N,nwindow", [(12000, 1500), (12345, 1500), (12250, 1500), (4000, 4000),
                                      (6000, 200)])
def test_windows_match_oracle(gpu, oracle, N, nwindow, method):
    """auto: per-window harmonic moments (k_moments_win) — parity within the oracle's outcomes
    under 128-ulp χ² noise, as for the whole-exposure harmonic path; windows (and a last
    window) shorter than 256 samples are fitted exactly; exact: 1-ulp envelope."""
    B = exposure(N, seed=5)
    got, out = gpu.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], nwindow,
                               want_output=True, method=method)
    ref, pert = oracle_windows(oracle, B, nwindow, B["fc_of_pixel"], ulps=ulps_for(method))
    assert got.shape == ref.shape == (-(-N // nwindow), 32)
    exact = (got["status"] & gpu.GPD_ST_EXACT) != 0
    if method == "exact" or nwindow < 256:
        assert np.all(exact)
    else:
        spans = np.minimum(nwindow, N - nwindow * np.arange(got.shape[0]))
        assert np.all(exact[spans < 256])  # short last window: exact fallback
        assert np.mean(~exact[spans >= 256]) > 0.9  # harmonic fits
    if method == "exact":
        print(assert_exact_bitwise(got.reshape(-1), ref.reshape(-1),
                                   label=f"windows exact N={N} w={nwindow}"))
    else:
        # windows shorter than 256 samples (and a short last window) are fitted exactly: bitwise
        sp = np.minimum(nwindow, N - nwindow * np.arange(got.shape[0]))
        print(assert_exact_bitwise(got[sp < 256].reshape(-1), ref[sp < 256].reshape(-1),
                                   label="short windows"))
        # every harmonic window (≥ 256 samples) lands near NEWUOA's rhoend (1e-3) of the
        # oracle: tools/window_sweep.py (4 exposures of 8 windows × 32 diodes per length,
        # synth.make_batch(8·w, 32, seed=100..103), 12 draws at 128 ulp) measured max deviations
        # 6.2e-4 / 5.6e-4 / 5.1e-4 / 2.3e-4 / 4.1e-5 at w = 256 / 300 / 345 / 400 / 500, and
        # 1.5e-3 at w = 200 — windows below 256 samples are fitted exactly
        # (profiles/r3/window_sweep.json).  One sweep pins the bound, so windows below 400
        # samples keep a 3x margin (2e-3; advisor r3), the longer ones 1e-3.
        bound = 2e-3 if nwindow < 400 else 1e-3
        print(assert_fit_parity(got[sp >= 256].reshape(-1), ref[sp >= 256].reshape(-1),
                                [p[sp >= 256].reshape(-1) for p in pert],
                                label=f"windows {method} N={N} w={nwindow}", max_dev=bound)
              if np.any(sp >= 256) else "no harmonic windows")
    # output rows of window w use window w's parameters (src/GPPupilDemodulation.jl:207)
    for w in range(ref.shape[0]):
        I = slice(w * nwindow, min(N, (w + 1) * nwindow))
        _, refout = oracle.fit_batch(B["t"][I], B["d"][:, I], B["fc"][:, I], B["fc_of_pixel"],
                                     want_output=True)
        same = np.abs(got["b"][w] - ref["b"][w]) <= 1e-10 * ref["b"][w]
        assert np.max(np.abs(out[same][:, I] - refout[same])) <= 1e-9 * np.abs(B["d"]).max()


@pytest.mark.parametrize("method", ["auto", "exact"])
@pytest.mark.parametrize("onlyhigh", [False, True])
def test_windows_faint(gpu, oracle, onlyhigh, method):
    """Per-window compute_mean_var_power on state[I] (faint mode, :205)."""
    N, nwindow = 9000, 3000
    B = exposure(N, seed=23)
    st = faint_states(N, seed=3)
    power = np.where(st == 3, 1.1, np.where(st == 1, 0.3, 0.6))
    B["d"] = B["d"] * power[None, :]
    got = gpu.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], nwindow, state=st,
                          onlyhigh=onlyhigh, method=method)
    flags = oracle.RECENTER | (oracle.ONLY_HIGH if onlyhigh else 0)
    ref, pert = oracle_windows(oracle, B, nwindow, B["fc_of_pixel"], state=st, flags=flags,
                               ulps=ulps_for(method))
    if method == "exact":
        print(assert_exact_bitwise(got.reshape(-1), ref.reshape(-1),
                                   label=f"faint windows exact onlyhigh={onlyhigh}"))
        return
    print(assert_fit_parity(got.reshape(-1), ref.reshape(-1), [p.reshape(-1) for p in pert],
                            label=f"faint windows {method} onlyhigh={onlyhigh}"))


def test_windows_offsets_and_multi_gpu_split(gpu, oracle):
    N, nwindow = 6000, 1000
    B = synth.make_batch(N, 32, seed=9, offsets=True)
    got = gpu.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], nwindow, fitoffsets=True,
                          n_gpus=8)  # clamps to the visible devices
    # windows with fitoffsets are fitted by the exact evaluator: the oracle's bits per window
    ref, _ = oracle_windows(oracle, B, nwindow, B["fc_of_pixel"],
                            flags=oracle.RECENTER | oracle.FIT_OFFSETS, ulps=4.0)
    print(assert_exact_bitwise(got.reshape(-1), ref.reshape(-1), label="offsets windows"))


def test_windows_harmonic_offsets_rejected(gpu):
    B = synth.make_batch(2000, 4, seed=2)
    with pytest.raises(gpu.GpdError):
        gpu.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], 500, fitoffsets=True,
                        method="harmonic")


def test_demodulate_windows_api(gpu, oracle):
    """The 40-column exposure API: output, per-window records and the Float32 tables."""
    N = 5000
    B = exposure(N, seed=42)
    data = np.empty((N, 40), dtype=np.complex128)
    data[:, :32] = B["d"].T
    fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)])
    for g in range(8):
        cols = np.nonzero(fop == 32 + g)[0]
        data[:, 32 + g] = B["fc"][B["fc_of_pixel"][cols[0]]]
    window_s = 2.0  # 1000 samples at 500 Hz
    output, params, tables = gpu.demodulate_windows(B["t"], data, window_s)
    nw = gpu.window_length(B["t"], window_s)
    assert nw == 1000 and params.shape == (5, 32)
    np.testing.assert_array_equal(output[:, 32:], data[:, 32:])
    assert tables["B"].shape == (32, N)
    np.testing.assert_array_equal(tables["B"][:, 1500], params["b"][1].astype(np.float32))
    ref0 = oracle.fit_batch(B["t"][:nw], data[:nw, :32].T, data[:nw].T, fop)
    ok = np.abs(params["b"][0] - ref0["b"]) <= 1e-10 * ref0["b"]
    assert ok.mean() >= 0.7


@pytest.mark.parametrize("faint,fitoffsets", [(False, False), (True, False), (False, True)])
def test_short_windows_one_wave_per_series(gpu, oracle, opts, faint, fitoffsets):
    """Windows of < 256 samples are fitted exactly; past two 256-thread workgroups per CU of them
    the library takes one wave per series (k_fit_exact WGT = 64, which reduces a canonical block
    as block_sum's four waves would).  Its records equal the 256-thread kernel's byte for byte
    and the oracle's on every window slice bit for bit (1 200 series of 40 samples, with a
    ragged last window)."""
    N, w = 3013, 40
    B = synth.make_batch(N, 16, seed=77, offsets=fitoffsets)
    st = faint_states(N, seed=3) if faint else None
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"], w)
    kw = dict(state=st, fitoffsets=fitoffsets, method="exact")
    opts("exact_wgt", 0)
    auto = gpu.fit_windows(*args, **kw)
    assert auto.size > 2 * 256  # the one-wave kernel's range on a 256-CU part
    opts("exact_wgt", 256)
    wg256 = gpu.fit_windows(*args, **kw)
    assert auto.tobytes() == wg256.tobytes()
    flags = oracle.RECENTER | (oracle.FIT_OFFSETS if fitoffsets else 0)
    ref = np.stack([oracle.fit_batch(B["t"][I], B["d"][:, I], B["fc"][:, I], B["fc_of_pixel"],
                                     state=None if st is None else st[I], flags=flags)
                    for I in (slice(s0, min(N, s0 + w)) for s0 in range(0, N, w))])
    print(assert_exact_bitwise(auto.reshape(-1), ref.reshape(-1),
                               label=f"one wave per series, faint={faint} offsets={fitoffsets}"))
