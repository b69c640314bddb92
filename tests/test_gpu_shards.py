"""Sharding is invisible in the results (BASELINE C4).

Series are independent (src/Modulation.jl:387-389), so a batch split over devices must give the
1-device records bit for bit.  The harmonic moments are sums over fixed sample units (a function
of N only), so neither the shard a series lands in nor the moment grid's fill (units per
workgroup, option upw) changes them.  Option fake_gpus = 1 keeps n_gpus shards on a one-GPU box (shard g
on device g % ndev): the library's multi-device split — series or window ranges, per-shard FC
column subsets, record and output offsets — runs here exactly as on an 8-GPU node."""
import numpy as np
import pytest

import synth
from test_gpu_parity import faint_states

pytestmark = pytest.mark.gpu


def _same(a, b):
    ra = a.view(np.uint8).reshape(len(a), -1)
    rb = b.view(np.uint8).reshape(len(b), -1)
    diff = int((ra != rb).any(axis=1).sum())
    assert diff == 0, f"{diff}/{len(a)} records differ"


@pytest.mark.parametrize("method", ["auto", "exact"])
@pytest.mark.parametrize("faint", [False, True])
def test_fit_batch_shards_bit_identical(gpu, opts, method, faint):
    opts("fake_gpus", 1)
    N, P = 5003, 70  # ragged: P not a multiple of 4 or of the shard count
    B = synth.make_batch(N, P, seed=61)
    st = faint_states(N, seed=3) if faint else None
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    ref, ref_out = gpu.fit_batch(*args, state=st, method=method, want_output=True)
    for g in (2, 3, 8):
        got, out = gpu.fit_batch(*args, state=st, method=method, want_output=True, n_gpus=g)
        _same(got, ref)
        np.testing.assert_array_equal(out, ref_out)


def test_fit_batch_shards_offsets_harmonic(gpu, opts):
    """Harmonic fitoffsets: the shards' FC-column subsets carry their own G_n moments."""
    opts("fake_gpus", 1)
    B = synth.make_batch(4000, 48, seed=62, offsets=True)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    ref = gpu.fit_batch(*args, fitoffsets=True, method="harmonic")
    for g in (2, 5):
        _same(gpu.fit_batch(*args, fitoffsets=True, method="harmonic", n_gpus=g), ref)


@pytest.mark.parametrize("window", [1500, 200])
def test_fit_windows_shards_bit_identical(gpu, opts, window):
    """Windows are split over devices (not diodes): a ragged last window, window-major record
    offsets and the demodulated output slices must land where the 1-device call puts them."""
    opts("fake_gpus", 1)
    N = 12_345
    B = synth.make_batch(N, 32, seed=63)
    fop = np.arange(32) // 4
    ref, ref_out = gpu.fit_windows(B["t"], B["d"], B["fc"], fop, window, want_output=True)
    for g in (2, 3):
        got, out = gpu.fit_windows(B["t"], B["d"], B["fc"], fop, window, want_output=True,
                                   n_gpus=g)
        _same(got, ref)
        np.testing.assert_array_equal(out, ref_out)


def _exposure(gpu, N, seed):
    B = synth.make_batch(N, 32, seed=seed)
    data = np.empty((40, N), dtype=np.complex128)
    data[:32] = B["d"]
    fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)])
    for g in range(8):
        data[32 + g] = B["fc"][B["fc_of_pixel"][np.nonzero(fop == 32 + g)[0][0]]]
    return B["t"], data.T


@pytest.mark.parametrize("storage", ["c64", "c32"])
def test_demodulateall_shards_bit_identical(gpu, opts, storage):
    """gpd_demodulateall over 2, 3 and 8 shards (advisor r5): each shard writes its slice of the
    32 demodulated columns through the staging ring (shards on one device take turns), the FC
    columns are copied beside them — output (every column, FC included), records and likelihood
    equal the 1-device call's bits, for ComplexF64 and ComplexF32 exposures."""
    opts("fake_gpus", 1)
    t, data = _exposure(gpu, 20_011, 64)
    if storage == "c32":
        data = np.asfortranarray(data.astype(np.complex64))
    out1, par1, lk1 = gpu.demodulateall(t, data)
    assert out1.dtype == data.dtype
    np.testing.assert_array_equal(out1[:, 32:], data[:, 32:])
    for g in (2, 3, 8):
        out, par, lk = gpu.demodulateall(t, data, n_gpus=g)
        np.testing.assert_array_equal(out, out1)
        np.testing.assert_array_equal(lk, lk1)
        assert [(p.a, p.b, p.ϕ) for p in par] == [(p.a, p.b, p.ϕ) for p in par1]


def test_demodulateall_pageable_staging_and_long_exposure(gpu, opts):
    """The staging ring is bounded (4 × 16 MB per device, advisor r5): an exposure whose
    demodulated columns exceed it (32 × 200 000 × 16 B = 102 MB: 7 chunks through 4 slots) gives
    the same output as the fit-batch path; and the pageable ring — what runs when pinning fails
    (option stage_pinned = 0 forces it) — gives the same bytes as the pinned one."""
    t, data = _exposure(gpu, 200_000, 65)
    out, par, lk = gpu.demodulateall(t, data)
    cols = np.ascontiguousarray(data.T)
    fop = np.array([gpu.fc_column_of(c) - 1 for c in range(1, 33)], dtype=np.int32)
    ref, ref_out = gpu.fit_batch(t, cols[:32], cols, fop, want_output=True)
    np.testing.assert_array_equal(out[:, :32].T, ref_out)
    np.testing.assert_array_equal(lk, ref["chi2"])
    opts("stage_pinned", 0)
    out2, _, lk2 = gpu.demodulateall(t, data)
    np.testing.assert_array_equal(out2, out)
    np.testing.assert_array_equal(lk2, lk)
    d32 = np.asfortranarray(data.astype(np.complex64))
    o32, _, _ = gpu.demodulateall(t, d32)
    opts("stage_pinned", 1)
    o32p, _, _ = gpu.demodulateall(t, d32)
    np.testing.assert_array_equal(o32, o32p)


def test_records_independent_of_batch_and_grid(gpu, opts):
    """A series' harmonic record does not depend on the other series of its batch (a sub-batch
    starting mid-workgroup) nor on the moment grid (units per workgroup 1, 2, 3, 7)."""
    N, P = 20_000, 96
    B = synth.make_batch(N, P, seed=64)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    ref = gpu.fit_batch(*args, method="harmonic")
    sub = slice(36, 84)
    fo = B["fc_of_pixel"][sub]
    got = gpu.fit_batch(B["t"], B["d"][sub], B["fc"][fo.min():fo.max() + 1], fo - fo.min(),
                        method="harmonic")
    _same(got, ref[sub])
    for upw in ("1", "2", "3", "7"):
        opts("upw", int(upw))
        _same(gpu.fit_batch(*args, method="harmonic"), ref)


def test_full_length_shard_invariance_device(gpu):
    """At the full exposure length (N = 1e5, the C3/C4 series) on device buffers: the records of
    a 512-series shard taken from the middle of a 2048-series batch (offset 1024, as rank 2 of 4
    would hold it) equal the batch's own records for those series, bit for bit — the C4 split's
    property at C4's series length, through gpd_fit_batch_dev."""
    import ctypes
    import torch
    L = gpu.load()
    dev = torch.device("cuda", 0)
    sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    N, P = 100_000, 2048
    t = torch.empty(N, dtype=torch.float64, device=dev)
    d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
    fc = torch.empty((P // 4, N, 2), dtype=torch.float64, device=dev)
    fcop = torch.empty(P, dtype=torch.int32, device=dev)
    gpu._lib.check(L.gpd_synth_fill_dev(N, P, 0, 7, 0.0, 0.002, 0.1, 0, gpu.M_2PI, t.data_ptr(),
                                        d.data_ptr(), N, fc.data_ptr(), N, fcop.data_ptr(), None,
                                        0, sptr))
    err = ctypes.create_string_buffer(512)

    def fit(p0, p1):
        out = torch.empty((p1 - p0, 64), dtype=torch.uint8, device=dev)
        fo = (fcop[p0:p1] - p0 // 4).contiguous()
        gpu._lib.check(L.gpd_fit_batch_dev(N, p1 - p0, t.data_ptr(), d[p0].data_ptr(), N,
                                           fc[p0 // 4].data_ptr(), (p1 - p0) // 4, N,
                                           fo.data_ptr(), None, gpu.M_2PI, None,
                                           gpu.GPD_RECENTER, 60, out.data_ptr(), None, N, 0,
                                           sptr, err, len(err)), err)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy().reshape(-1).view(gpu.PARAM_DTYPE)

    whole = fit(0, P)
    _same(fit(1024, 1536), whole[1024:1536])
    assert not np.any(whole["status"] & gpu.GPD_ST_NAN)


@pytest.mark.parametrize("faint", [False, True])
@pytest.mark.parametrize("storage", ["c64", "c32"])
def test_cohort_pipeline_records_bitwise(gpu, opts, faint, storage):
    """The pipelined harmonic path (series cohorts: moments of cohort c on the caller's stream
    while cohort c−1's fit runs on the side stream, gpd_engine.hip) gives the one-cohort records
    bit for bit, for any cohort count — the fixed sample units make a series' moments
    independent of the cohort it is in, including a ragged last cohort."""
    import synth
    from test_gpu_parity import faint_states
    N, P = 12_000, 1000
    B = synth.make_batch(N, P, seed=21)
    st = None
    if faint:
        st = faint_states(N, seed=6)
        B["d"] = B["d"] * np.where(st == 3, 1.1, np.where(st == 1, 0.05, 0.3))[None, :]
    d, fc = B["d"], B["fc"]
    if storage == "c32":
        d, fc = d.astype(np.complex64), fc.astype(np.complex64)
    args = (B["t"], d, fc, B["fc_of_pixel"])
    recs = {}
    opts("h2d_parts", 1)  # one device pipeline over the whole batch (parts would be cohorts' size)
    for c in ("1", "2", "3", "5"):
        opts("cohorts", int(c))
        recs[c] = gpu.fit_batch(*args, state=st, method="harmonic")
    for c, r in recs.items():
        _same(r, recs["1"])
    assert not np.any(recs["1"]["status"] & gpu.GPD_ST_NAN)
    opts("cohorts", 2)
    gpu.fit_batch(*args, state=st, method="harmonic")
    t = gpu.timings(0)
    assert "fit_tail" in t and t["moments"] > 0, t  # the cohort path ran


@pytest.mark.parametrize("storage", ["c64", "c32"])
def test_cu_masked_streams_records_bitwise(gpu, opts, storage):
    """The CU-masked A/B paths (options mom_cus: the moment pass on a stream masked to n CUs;
    fit_cus with cohorts: the fits of all but the last cohort on r CUs per XCD, the moments on the
    others — DESIGN.md §15) give the default path's records bit for bit, c64 and c32."""
    N, P = 12_000, 1000
    B = synth.make_batch(N, P, seed=23)
    d, fc = B["d"], B["fc"]
    if storage == "c32":
        d, fc = d.astype(np.complex64), fc.astype(np.complex64)
    args = (B["t"], d, fc, B["fc_of_pixel"])
    opts("h2d_parts", 1)
    ref = gpu.fit_batch(*args, method="harmonic")
    for setting in ({"mom_cus": 192}, {"mom_cus": 248}, {"cohorts": 3, "fit_cus": 2},
                    {"cohorts": 5, "fit_cus": 1}):
        for k, v in setting.items():
            opts(k, v)
        _same(gpu.fit_batch(*args, method="harmonic"), ref)
        for k in setting:
            opts(k, 0 if k != "cohorts" else 1)


def test_series_per_fit_wave_does_not_change_records(gpu, opts):
    """The harmonic fit's shape follows the batch (fit_shape, gpd_engine.hip): lanes per series
    (1, 2, 4, 8 — the objective's harmonic slots and NEWUOA's 49-angle searches split across
    them), series per wave and waves per workgroup.  The objective's arithmetic is canonical and
    the split angle searches pick the sequential loop's index and values, so the records are the
    same bytes for every shape and for the automatic choice (C2-sized batch and a batch that
    fills several waves per CU), the exact fallback and the π-flip re-fits included."""
    fallbacks = 0
    for N, P in ((20_000, 32), (8_000, 700)):
        B = synth.make_batch(N, P, seed=N + P, b_range=(0.3, 5.5))  # b > 4.5: exact fallback
        args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
        gpu.reset_options()
        ref = gpu.fit_batch(*args, method="auto")
        fallbacks += int(np.count_nonzero(ref["status"] & gpu.GPD_ST_FALLBACK))
        for lps, lanes, wpb in ((1, 1, 1), (1, 7, 4), (1, 64, 1), (1, 49, 4), (2, 1, 1),
                                (2, 32, 4), (4, 3, 2), (4, 16, 4), (8, 1, 1), (8, 8, 4),
                                (8, 5, 3)):
            opts("fit_lps", lps)
            opts("fit_lanes", lanes)
            opts("fit_wpb", wpb)
            _same(gpu.fit_batch(*args, method="auto"), ref)
        assert np.mean((ref["status"] & gpu.GPD_ST_EXACT) == 0) > 0.5  # mostly harmonic
    # the fallback path is part of the comparison (whether NEWUOA probes |b| > 4.5 depends on
    # its trajectory: the 700-series batch mostly stops at maxfun below b ≈ 4.5, as the
    # oracle's own fits do)
    assert fallbacks > 0


def test_fit_moment_source_does_not_change_records(gpu, opts):
    """With several lanes per series the harmonic fit reads each series' moments (and, with
    fitoffsets, its FC column's) from a copy in LDS (option fit_mcache, default 1) instead of
    L2: the same values, so the same records, for every multi-lane shape, with and without
    fitoffsets (r5)."""
    N, P = 20_000, 64
    B = synth.make_batch(N, P, seed=5, b_range=(0.3, 4.0))
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    for offs in (False, True):
        for lps, lanes, wpb in ((2, 8, 1), (4, 3, 2), (4, 16, 4), (8, 1, 1), (8, 8, 4)):
            gpu.reset_options()
            opts("fit_lps", lps)
            opts("fit_lanes", lanes)
            opts("fit_wpb", wpb)
            a = gpu.fit_batch(*args, method="harmonic", fitoffsets=offs)
            opts("fit_mcache", 0)
            b = gpu.fit_batch(*args, method="harmonic", fitoffsets=offs)
            _same(a, b)


def test_flip_refits_same_records_in_every_fit_shape(gpu, opts):
    """A batch where ~1 % of the series land in a "bad minimum" and are re-fitted from ϕ ∓ π
    (src/Modulation.jl:411-414; large b, noisy): every fit shape — one lane per series in one or
    several rounds of waves, several lanes per series — gives the automatic shape's records,
    re-fits included, with and without fitoffsets (r5)."""
    N, P = 2000, 2048
    B = synth.make_batch(N, P, seed=3, b_range=(0.3, 4.0), sigma=0.5)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    for offs in (False, True):
        gpu.reset_options()
        ref = gpu.fit_batch(*args, method="harmonic", fitoffsets=offs)
        assert int(((ref["status"] & 1) != 0).sum()) >= 5  # GPD_ST_REFIT
        for lps, lanes in ((1, 64), (1, 3), (1, 1), (4, 16), (8, 1)):
            gpu.reset_options()
            opts("fit_lps", lps)
            opts("fit_lanes", lanes)
            _same(gpu.fit_batch(*args, method="harmonic", fitoffsets=offs), ref)


def test_faint_state_pointer_alignment(gpu):
    """The state-split faint moments read each tile's 32 state bytes in 16-B loads only when the
    caller's state array is 16-B aligned (k_faint_defer); a state view at an odd byte offset
    takes the byte path and must give the same records, bit for bit (device buffers)."""
    import ctypes
    import torch
    L = gpu.load()
    dev = torch.device("cuda", 0)
    sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    N, P = 20_000, 64
    t = torch.empty(N, dtype=torch.float64, device=dev)
    d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
    fc = torch.empty((P // 4, N, 2), dtype=torch.float64, device=dev)
    fcop = torch.empty(P, dtype=torch.int32, device=dev)
    gpu._lib.check(L.gpd_synth_fill_dev(N, P, 0, 9, 0.0, 0.002, 0.1, 0, gpu.M_2PI, t.data_ptr(),
                                        d.data_ptr(), N, fc.data_ptr(), N, fcop.data_ptr(), None,
                                        0, sptr))
    rng = np.random.default_rng(3)
    st = np.empty(N, np.int8)
    i = 0
    while i < N:  # runs of 1..60 samples: most tiles hold several valid states
        n = int(rng.integers(1, 61))
        st[i:i + n] = rng.choice([-1, 1, 2, 3], p=[0.1, 0.3, 0.3, 0.3])
        i += n
    err = ctypes.create_string_buffer(512)

    def fit(state_dev):
        out = torch.empty((P, 64), dtype=torch.uint8, device=dev)
        gpu._lib.check(L.gpd_fit_batch_dev(N, P, t.data_ptr(), d.data_ptr(), N, fc.data_ptr(),
                                           P // 4, N, fcop.data_ptr(), state_dev.data_ptr(),
                                           gpu.M_2PI, None, gpu.GPD_RECENTER, 60, out.data_ptr(),
                                           None, N, 0, sptr, err, len(err)), err)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy().reshape(-1).view(gpu.PARAM_DTYPE)

    aligned = torch.from_numpy(st).to(dev)
    buf = torch.zeros(N + 16, dtype=torch.int8, device=dev)
    odd = buf[3:3 + N]
    odd.copy_(aligned)
    assert odd.data_ptr() % 16 == 3
    a, b = fit(aligned), fit(odd)
    _same(b, a)
    assert not np.all(a["status"] & gpu.GPD_ST_NAN)



@pytest.mark.parametrize("faint", [False, True])
def test_h2d_parts_bit_identical(gpu, opts, faint):
    """Host-buffer harmonic calls cut into parts (option h2d_parts, r6: part k's columns cross
    PCIe on a copy stream while part k−1 computes, the staged output returns on a third stream)
    give the one-part call's records, output and faint statistics bit for bit — for a ragged
    batch (P = 70: parts at multiples of 4, a short last part), for parts inside device shards,
    and for the exact method (which never splits)."""
    N, P = 5003, 70
    B = synth.make_batch(N, P, seed=66)
    st = faint_states(N, seed=5) if faint else None
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    opts("h2d_parts", 1)
    ref, ref_out = gpu.fit_batch(*args, state=st, want_output=True)
    ref_fs = gpu.last_faint_stats(P) if faint else None
    for parts in (2, 3, 4, 8):
        opts("h2d_parts", parts)
        got, out = gpu.fit_batch(*args, state=st, want_output=True)
        _same(got, ref)
        np.testing.assert_array_equal(out, ref_out)
        if faint:
            for a, b in zip(gpu.last_faint_stats(P), ref_fs):
                np.testing.assert_array_equal(a, b)
    opts("fake_gpus", 1)
    opts("h2d_parts", 3)
    got, out = gpu.fit_batch(*args, state=st, want_output=True, n_gpus=2)
    _same(got, ref)
    np.testing.assert_array_equal(out, ref_out)


@pytest.mark.parametrize("storage", ["c64", "c32"])
def test_demodulateall_h2d_parts_bit_identical(gpu, opts, storage):
    """gpd_demodulateall with its H2D, compute and staged D2H pipelined over 1, 2, 4 and 8 parts:
    every output column (FC included), record and likelihood equal across part counts — also for
    an exposure whose demodulated columns exceed the staging ring (200 000 samples: each part's
    chunks cycle through the 4 slots)."""
    for N, seed in ((20_011, 67), (200_000, 68)):
        t, data = _exposure(gpu, N, seed)
        if storage == "c32":
            data = np.asfortranarray(data.astype(np.complex64))
        opts("h2d_parts", 1)
        out1, par1, lk1 = gpu.demodulateall(t, data)
        for parts in (2, 4, 8):
            opts("h2d_parts", parts)
            out, par, lk = gpu.demodulateall(t, data)
            np.testing.assert_array_equal(out, out1)
            np.testing.assert_array_equal(lk, lk1)
            assert [(p.a, p.b, p.ϕ) for p in par] == [(p.a, p.b, p.ϕ) for p in par1]
