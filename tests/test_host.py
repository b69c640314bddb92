"""CPU checks of the host-side mirror (idx/Side/Diode/MetState, FaintStates, argument handling)
and of the multi-GPU sharding helpers."""
import os

import numpy as np
import pytest


def test_idx_matches_reference_layout(gpd):
    """src/Modulation.jl:17-22: FT T1..T4 D1..D4 → 1..16, SC → 17..32, FC FT → 33..36, FC SC → 37..40."""
    S, D = gpd.Side, gpd.Diode
    assert gpd.idx(S.FT, 1, D.D1) == 1
    assert gpd.idx(S.FT, 4, D.D4) == 16
    assert gpd.idx(S.SC, 1, D.D1) == 17
    assert gpd.idx(S.SC, 4, D.D4) == 32
    assert [gpd.idx(S.FT, t, D.FC) for t in range(1, 5)] == [33, 34, 35, 36]
    assert [gpd.idx(S.SC, t, D.FC) for t in range(1, 5)] == [37, 38, 39, 40]
    cols = sorted(gpd.idx(s, t, d) for s in S for t in range(1, 5) for d in D)
    assert cols == list(range(1, 41))
    for c in range(1, 33):
        side = S.FT if c <= 16 else S.SC
        tel = (c - 1) % 16 // 4 + 1
        assert gpd.fc_column_of(c) == gpd.idx(side, tel, D.FC)


def test_metstate_codes(gpd):
    M = gpd.MetState
    assert (M.OFF, M.LOW, M.NORMAL, M.HIGH, M.TRANSIENT) == (0, 1, 2, 3, -1)


def test_faintstates_orders_by_voltage(gpd):
    fs = gpd.FaintStates.make([1.0, 2.0], [1.5], 5.0, 1.0)  # voltage1 > voltage2 → swap
    np.testing.assert_array_equal(fs.timer1, [1.5])
    np.testing.assert_array_equal(fs.timer2, [1.0, 2.0])
    assert (fs.state1, fs.state2) == (gpd.MetState.HIGH, gpd.MetState.LOW)


def test_demodulateall_validates_like_reference(gpd):
    t = np.arange(100) * 0.002
    with pytest.raises(TypeError):
        gpd.demodulateall(t, np.zeros((100, 40)))            # not complex
    with pytest.raises(ValueError):
        gpd.demodulateall(t, np.zeros((100, 39), complex))   # not N×40
    with pytest.raises(ValueError):
        gpd.demodulateall(t[:99], np.zeros((100, 40), complex))
    with pytest.raises(ValueError):
        gpd.demodulateall(t, np.zeros((100, 40), complex), faintparam=np.zeros(7, np.int8))


def test_shard_range_partitions_whole_groups(gpd):
    from gpdemod import shard

    for n, w in [(100_000, 8), (32, 8), (40, 3), (7, 2), (1, 4)]:
        spans = [shard.shard_range(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        for (a, b), (c, _) in zip(spans, spans[1:]):
            assert b == c and a <= b
        assert all(a % 4 == 0 for a, _ in spans)
    assert shard.weak_offset(100_000, 3) == 300_000
    with pytest.raises(ValueError):
        shard.weak_offset(10, 1)


def test_read_stefan_file_fixture(gpd):
    """The reference's own calibration data (data/Stefan_file.txt, copied to tests/golden/):
    40 `avg` rows → 40 centres at idx(side, telescope, diode) (src/GPPupilDemodulation.jl:88-104)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "Stefan_file.txt")
    with open(path) as f:
        n_avg = sum(1 for line in f if line.startswith("avg"))
    assert n_avg == 40
    c = gpd.read_stefan_file(path)
    assert c.shape == (40,) and np.all(c != 0)
    k = gpd.idx(gpd.Side.FT, 1, gpd.Diode.FC) - 1  # "avg FTT1FC 0.5056591585058203 … 0.6414248583206548"
    assert c[k] == 1e-3 * (0.5056591585058203 + 1j * 0.6414248583206548)
    k = gpd.idx(gpd.Side.FT, 1, gpd.Diode.D1) - 1  # "avg FTT1D1 -3.9217663072871978 … -5.375368693370768"
    assert c[k] == 1e-3 * (-3.9217663072871978 - 1j * 5.375368693370768)


def test_process_volt_argument_checks(gpd):
    t = np.arange(100) * 0.002
    with pytest.raises(ValueError):
        gpd.process_volt(t, np.zeros((100, 79), np.float32))
    with pytest.raises(NotImplementedError):
        gpd.process_volt(t, np.zeros((100, 80), np.float32), offsets=True)


def test_buildfaintparameters_from_header(gpd):
    """src/GPPupilDemodulation.jl:64-81: timers from TIMERi/RATEi/REPEATi, ordered by voltage."""
    hdr = {"MJD-OBS": 60000.5, "ESO INS ANLO3 RATE1": 11.0, "ESO INS ANLO3 RATE2": 11.0,
           "ESO INS ANLO3 REPEAT1": 5, "ESO INS ANLO3 REPEAT2": 4,
           "ESO INS ANLO3 TIMER1": 1.7e9, "ESO INS ANLO3 TIMER2": 1.7e9 + 1.0,
           "ESO INS ANLO3 VOLTAGE1": 4.5, "ESO INS ANLO3 VOLTAGE2": 1.0}
    fs = gpd.buildfaintparameters(hdr)
    off = 40587.0 * 86400
    # voltage1 > voltage2: timer1 is the LOW one, so the structure swaps them (src/Faint.jl:14-16)
    np.testing.assert_array_equal(fs.timer1, 1.7e9 + 1.0 + off + 11.0 * np.arange(4))
    np.testing.assert_array_equal(fs.timer2, 1.7e9 + off + 11.0 * np.arange(5))
    assert (fs.voltage1, fs.voltage2) == (1.0, 4.5)
    t = gpd.metrology_times(np.array([0, 2000, 4000], dtype=np.int64), 60000.5)
    np.testing.assert_array_equal(t, np.array([0, 2000, 4000]) * 1e-6 + 86400 * 60000.5)
