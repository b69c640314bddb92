"""GPU: processmetrology's numeric core straight from Float32 VOLT rows (§8f rank 3) —
ingest (Float64.(VOLT), centring), demodulateall / windows, egress to Float32 rows."""
import numpy as np
import pytest

import synth
from test_gpu_parity import assert_exact_bitwise, assert_fit_parity, perturbed_runs

pytestmark = pytest.mark.gpu


def volt_exposure(gpu, N, seed):
    B = synth.make_batch(N, 32, seed=seed)
    data = np.empty((N, 40), dtype=np.complex128)
    data[:, :32] = B["d"].T
    fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)])
    for g in range(8):
        cols = np.nonzero(fop == 32 + g)[0]
        data[:, 32 + g] = B["fc"][B["fc_of_pixel"][cols[0]]]
    rng = np.random.default_rng(seed)
    centres = 0.05 * (rng.standard_normal(40) + 1j * rng.standard_normal(40))
    raw = data + centres[None, :]  # what the instrument records before centring
    volt = np.empty((N, 80), dtype=np.float32)
    volt[:, 0::2] = raw.real
    volt[:, 1::2] = raw.imag
    cplx = volt[:, 0::2].astype(np.float64) + 1j * volt[:, 1::2].astype(np.float64)
    return B["t"], volt, centres, cplx - centres[None, :], fop


def test_process_volt_matches_oracle(gpu, oracle):
    t, volt, centres, cplx, fop = volt_exposure(gpu, 20000, seed=17)
    out, params, tables = gpu.process_volt(t, volt, offsets=centres)
    assert tables is None and params.shape == (32,)
    ref, refout = oracle.fit_batch(t, cplx[:, :32].T, cplx.T, fop, want_output=True)
    B = {"t": t, "d": np.ascontiguousarray(cplx[:, :32].T), "fc": np.ascontiguousarray(cplx.T),
         "fc_of_pixel": fop}
    print(assert_fit_parity(params, ref, perturbed_runs(oracle, B, ulps=128.0), label="volt"))
    # egress: demodulated columns and centred FC columns as Float32 rows
    fc32 = cplx[:, 32:].astype(np.complex64)
    np.testing.assert_array_equal(out[:, 64::2], fc32.real)
    np.testing.assert_array_equal(out[:, 65::2], fc32.imag)
    same = np.abs(params["b"] - ref["b"]) <= 1e-10 * ref["b"]
    got = out[:, 0:64:2].astype(np.float64) + 1j * out[:, 1:64:2]
    ref32 = refout.T.astype(np.complex64)
    diff = np.abs(got[:, same] - ref32[:, same])
    assert diff.max() <= 2 * np.spacing(np.float32(np.abs(cplx).max()))  # ≤ Float32 rounding


def test_process_volt_windows_equal_fit_windows(gpu):
    t, volt, centres, cplx, fop = volt_exposure(gpu, 12000, seed=29)
    out, params, tables = gpu.process_volt(t, volt, offsets=centres, window=8.0)  # 4000 samples
    assert params.shape == (3, 32) and tables["PHI"].shape == (32, 12000)
    fw = gpu.fit_windows(t, cplx[:, :32].T, cplx.T, fop, 4000)
    np.testing.assert_array_equal(params["b"], fw["b"])  # same device pipeline, same inputs
    np.testing.assert_array_equal(params["chi2"], fw["chi2"])


def test_process_volt_fitoffsets_without_centring(gpu, oracle):
    t, volt, centres, cplx, fop = volt_exposure(gpu, 8000, seed=31)
    out, params, _ = gpu.process_volt(t, volt, offsets=False)  # fitoffsets, no centring (:155-157)
    raw = volt[:, 0::2].astype(np.float64) + 1j * volt[:, 1::2].astype(np.float64)
    ref = oracle.fit_batch(t, raw[:, :32].T, raw.T, fop, flags=oracle.RECENTER | oracle.FIT_OFFSETS)
    # fitoffsets takes the exact evaluator: the oracle's bits (the multi-workgroup split of a
    # 32-series exposure included)
    print(assert_exact_bitwise(params, ref, label="volt offsets"))


def test_processmetrology_table_and_header(gpu):
    """processmetrology (src/GPPupilDemodulation.jl:128-255) outputs: header keywords in the
    reference's order and names, VOLT rows (80, or 144 with keepraw), window-mode columns."""
    t, volt, centres, cplx, fop = volt_exposure(gpu, 6000, seed=37)
    table = {"TIME": np.round((t - t[0]) * 1e6).astype(np.int64), "VOLT": volt,
             "OTHER": np.arange(t.size)}
    header = {"MJD-OBS": 60123.25, "EXTNAME": "METROLOGY"}
    tab, hdr = gpu.processmetrology(table, header, offsets=centres)
    times = gpu.metrology_times(table["TIME"], 60123.25)
    out, params, _ = gpu.process_volt(times, volt, offsets=centres)
    np.testing.assert_array_equal(tab["VOLT"], out)
    assert tab["OTHER"] is table["OTHER"] and hdr["PROCSOFT"] == "GPPupilDemodulation.jl"
    keys = [k for k in hdr if k.startswith("DEMODULATION")]
    assert len(keys) == 4 * 32 and keys[:5] == [
        "DEMODULATION AMPLITUDE ABS FT T1 D1", "DEMODULATION AMPLITUDE ARG FT T1 D1",
        "DEMODULATION SIN AMPLITUDE FT T1 D1", "DEMODULATION SIN PHASE FT T1 D1",
        "DEMODULATION AMPLITUDE ABS FT T1 D2"]
    k = gpu.idx(gpu.Side.SC, 3, gpu.Diode.D2) - 1
    assert hdr["DEMODULATION SIN AMPLITUDE SC T3 D2"] == params["b"][k]
    assert hdr["DEMODULATION AMPLITUDE ARG SC T3 D2"] == np.angle(params["a"][k])
    # keepraw: raw rows first, then the 32 demodulated columns
    tab2, _ = gpu.processmetrology(table, header, offsets=centres, keepraw=True)
    assert tab2["VOLT"].shape == (t.size, 144)
    np.testing.assert_array_equal(tab2["VOLT"][:, :80], volt)
    np.testing.assert_array_equal(tab2["VOLT"][:, 80:], out[:, :64])
    # fitoffsets keywords, window columns + STATE
    _, hdr3 = gpu.processmetrology(table, header, offsets=False)
    assert "DEMODULATION CENTER X0 FT T1 D1" in hdr3
    highs = times[0] + np.array([2.0, 7.0])
    fs = gpu.FaintStates.make(highs, highs + 1.0, 1.0, 2.0)
    tab4, hdr4 = gpu.processmetrology(table, header, offsets=centres, window=4.0, faintparam=fs)
    assert not any(k.startswith("DEMODULATION") for k in hdr4)
    assert tab4["B"].shape == (t.size, 32) and tab4["B"].dtype == np.float32
    assert tab4["STATE"].dtype == np.int8 and set(np.unique(tab4["STATE"])) <= {-1, 1, 2, 3}


def test_processmetrology_fits_file(gpu, tmp_path):
    """processmetrology's (table, hdr) through the FITS writer and back (fits.py): the
    demodulated VOLT rows and window columns bit for bit, the DEMODULATION keywords to 15
    significant digits."""
    t, volt, centres, cplx, fop = volt_exposure(gpu, 6000, seed=41)
    table = {"TIME": np.round((t - t[0]) * 1e6).astype(np.int64), "VOLT": volt}
    header = {"MJD-OBS": 60123.25, "EXTNAME": "METROLOGY"}
    for kw in ({"offsets": False}, {"offsets": centres, "window": 4.0, "keepraw": True}):
        tab, hdr = gpu.processmetrology(table, header, **kw)
        path = str(tmp_path / "out.fits")
        gpu.fits.write_metrology(path, tab, hdr)
        (_, _), (h1, d1) = gpu.fits.read_fits(path)
        for k, a in tab.items():
            assert d1[k].tobytes() == np.ascontiguousarray(a).tobytes(), k
        for k, v in hdr.items():
            if k.startswith("DEMODULATION"):
                assert h1[k] == pytest.approx(v, rel=1e-14, abs=1e-300), k
        assert h1["PROCSOFT"] == "GPPupilDemodulation.jl"


def test_process_exposure_file(gpu, tmp_path):
    """The reference's per-file step (src/GPPupilDemodulation.jl:357-414): keyword gating, MJD-OBS
    from the primary header, METROLOGY replaced by processmetrology's table and header, the
    other HDUs copied."""
    t, volt, centres, cplx, fop = volt_exposure(gpu, 6000, seed=43)
    mjd = 60123.25
    times_us = np.round((t - t[0]) * 1e6).astype(np.int64)
    met_hdr = {"EXTNAME": "METROLOGY", "TTYPE1": "TIME", "TUNIT1": "us"}
    prim = {"ESO INS PMC1 MODULATE": True, "ESO INS MET MODE": "ON", "MJD-OBS": mjd}
    other = np.arange(12, dtype=np.float32).reshape(3, 4)
    src, dst = str(tmp_path / "exp.fits"), str(tmp_path / "exp_demod.fits")
    gpu.fits.write_fits(src, [(prim, None), ({"EXTNAME": "OTHER"}, other),
                              (met_hdr, {"TIME": times_us, "VOLT": volt})])
    assert gpu.process_exposure(src, dst, offsets=centres)
    out = gpu.fits.read_fits(dst)
    assert [h.get("EXTNAME") for h, _ in out] == [None, "OTHER", "METROLOGY"]
    np.testing.assert_array_equal(out[1][1], other)
    tab, hdr = gpu.processmetrology({"TIME": times_us, "VOLT": volt}, met_hdr, offsets=centres,
                                    mjd=mjd)
    h, d = out[2]
    assert d["VOLT"].tobytes() == tab["VOLT"].tobytes() and h["TUNIT1"] == "us"
    assert h["DEMODULATION SIN AMPLITUDE SC T3 D2"] == pytest.approx(
        hdr["DEMODULATION SIN AMPLITUDE SC T3 D2"], rel=1e-14)
    # gating: MODULATE false, MET MODE OFF → nothing written
    for bad in ({"ESO INS PMC1 MODULATE": False}, {"ESO INS MET MODE": "OFF"}):
        p2 = str(tmp_path / "skip.fits")
        gpu.fits.write_fits(p2, [(dict(prim, **bad), None), (met_hdr, {"TIME": times_us,
                                                                        "VOLT": volt})])
        assert not gpu.process_exposure(p2, str(tmp_path / "never.fits"), offsets=centres)
    assert not (tmp_path / "never.fits").exists()
