"""Device buildstates (gpd_buildstates_dev, gpd_states.hpp) against the host state machine
(gpd_buildstates) and the line-by-line transcription of src/Faint.jl:21-73 — bit-exact MetState
codes on the edge cases the reference loop has (entries closer than Δt, before t[0], at and after
t[N-1], repeated final timestamps, single entries, lag shifts, non-monotone timestamps)."""
import ctypes

import numpy as np
import pytest

from test_oracle import py_buildstates, random_timer_case

pytestmark = pytest.mark.gpu


def dev_buildstates(gpu, t, t1, t2, pre, post, lag=0):
    import torch

    L = gpu.load()
    td = torch.from_numpy(np.ascontiguousarray(t, dtype=np.float64)).cuda()
    st = torch.full((t.size,), 7, dtype=torch.int8, device="cuda")
    a1 = np.ascontiguousarray(t1, dtype=np.float64)
    a2 = np.ascontiguousarray(t2, dtype=np.float64)
    s = torch.cuda.current_stream()
    rc = L.gpd_buildstates_dev(t.size, td.data_ptr(), a1.size, a1.ctypes.data, a2.size,
                               a2.ctypes.data, int(lag), float(pre), float(post), st.data_ptr(),
                               0, ctypes.c_void_p(s.cuda_stream))
    gpu._lib.check(rc)
    torch.cuda.synchronize()
    return st.cpu().numpy()


def test_random_edge_cases(gpu):
    rng = np.random.default_rng(11)
    for _ in range(200):
        t, t1, t2, pre, post = random_timer_case(rng)
        got = dev_buildstates(gpu, t, t1, t2, pre, post)
        np.testing.assert_array_equal(got, py_buildstates(t, t1, t2, pre, post))


def test_exposure_scale_and_lag(gpu):
    """C5-like exposure (1e5 samples, HIGH 1 s per 11 s) with a lag shift, against the host."""
    t = 5.2e9 + np.arange(100_000) * 0.002
    highs = t[0] + np.arange(8.0, 190.0, 11.0)
    lows = highs + 1.0
    for lag in (0, -3, 4):
        fs = gpu.FaintStates.make(highs, lows, 1.0, 2.0)
        ref = gpu.buildstates(fs, t, lag=lag, preswitchdelay=0.01, postwitchdelay=0.3)
        got = dev_buildstates(gpu, t, highs, lows, 0.01, 0.3, lag=lag)
        np.testing.assert_array_equal(got, ref)


def test_non_monotone_timestamps_take_the_serial_loop(gpu):
    rng = np.random.default_rng(3)
    t = 1.0 + np.arange(3000) * 0.002
    t[1500:1510] = t[1500:1510][::-1]  # a local reversal
    t1 = np.sort(rng.uniform(t[0], t[-1], 6))
    t2 = np.sort(rng.uniform(t[0], t[-1], 5))
    got = dev_buildstates(gpu, t, t1, t2, 0.01, 0.05)
    np.testing.assert_array_equal(got, py_buildstates(t, t1, t2, 0.01, 0.05))


def test_states_feed_the_fit(gpu):
    """Device states straight into gpd_fit_batch: same fit as with the host-built states."""
    import synth

    B = synth.make_batch(6000, 8, seed=2)
    t = B["t"]
    highs = np.arange(1.0, 11.0, 2.2)
    lows = highs + 0.9
    fs = gpu.FaintStates.make(highs, lows, 1.0, 2.0)
    host = gpu.buildstates(fs, t, preswitchdelay=0.01, postwitchdelay=0.3)
    dev = dev_buildstates(gpu, t, highs, lows, 0.01, 0.3)
    np.testing.assert_array_equal(dev, host)
    a = gpu.fit_batch(t, B["d"], B["fc"], B["fc_of_pixel"], state=dev)
    b = gpu.fit_batch(t, B["d"], B["fc"], B["fc_of_pixel"], state=host)
    assert np.array_equal(a["b"], b["b"]) and np.array_equal(a["chi2"], b["chi2"])
