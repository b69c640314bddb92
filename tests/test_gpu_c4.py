"""BASELINE config C4 — the C3 batch (1e5 series × 1e5 samples, fp64) sharded over 8 GPUs — on
the path one rank of an 8-GPU node takes, run on the one-GPU test box.

Series are independent (src/Modulation.jl:387-389), so rank r of 8 fits the contiguous block
shard.shard_range(1e5, 8, r) (12 500 series, whole FC groups) with no data-path collective.  The
moment sums are cut into fixed sample units that depend on N only, so a shard's
records must equal the whole batch's records for those series BIT FOR BIT — whether the shard
is a view into the resident batch or, as bench.py's rank does, generated on its own device from
the counter RNG keyed by global series ids.  64 of the shard's series are also checked against
the CPU oracle with the harmonic evaluator's tie rule (test_gpu_parity.assert_fit_parity).

Device memory: the full batch is 200 GB (d 160 GB + FC 40 GB) of the 288 GB HBM; it is freed
before the shard is generated on its own.
"""
import ctypes

import numpy as np
import pytest

from test_gpu_parity import HARM_ULPS, assert_fit_parity

pytestmark = pytest.mark.gpu

N = 100_000
P = 100_000
WORLD, RANK = 8, 3
SEED = 7  # the C3/C4 seed


def test_c4_rank_shard_equals_full_batch(gpu, oracle):
    import torch

    from gpdemod import shard

    L = gpu.load()
    dev = torch.device("cuda", 0)
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    assert free > 215e9, f"C4 test needs ~215 GB of free HBM, {free / 1e9:.0f} GB free"
    sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    err = ctypes.create_string_buffer(512)
    p0, p1 = shard.shard_range(P, WORLD, RANK)
    assert (p0, p1) == (37_500, 50_000)
    n = p1 - p0

    def fit(nser, t, d_ptr, fc_ptr, n_fc, fcop):
        out = torch.empty((nser, 64), dtype=torch.uint8, device=dev)
        gpu._lib.check(L.gpd_fit_batch_dev(N, nser, t.data_ptr(), d_ptr, N, fc_ptr, n_fc, N,
                                           fcop.data_ptr(), None, gpu.M_2PI, None,
                                           gpu.GPD_RECENTER, 60, out.data_ptr(), None, N, 0,
                                           sptr, err, len(err)), err)
        torch.cuda.synchronize(dev)
        return out.cpu().numpy().reshape(-1).view(gpu.PARAM_DTYPE)

    # --- the whole C3 batch, resident ---------------------------------------------------
    t = torch.empty(N, dtype=torch.float64, device=dev)
    d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
    fc = torch.empty((P // 4, N, 2), dtype=torch.float64, device=dev)
    fcop = torch.empty(P, dtype=torch.int32, device=dev)
    gpu._lib.check(L.gpd_synth_fill_dev(N, P, 0, SEED, 0.0, 0.002, 0.1, 0, gpu.M_2PI,
                                        t.data_ptr(), d.data_ptr(), N, fc.data_ptr(), N,
                                        fcop.data_ptr(), None, 0, sptr))
    whole = fit(P, t, d.data_ptr(), fc.data_ptr(), P // 4, fcop)
    st = whole["status"]
    assert not np.any(st & (gpu.GPD_ST_NAN | gpu.GPD_ST_FALLBACK)), "C3 batch: NaN/fallback fits"

    # rank 3's shard as a view into the resident batch (d[p0], its own FC groups)
    fo = (fcop[p0:p1] - p0 // 4).contiguous()
    view = fit(n, t, d[p0].data_ptr(), fc[p0 // 4].data_ptr(), n // 4, fo)
    assert view.tobytes() == whole[p0:p1].tobytes(), "shard view: records differ from the batch"

    # 64 series of the shard (16 whole FC groups spread over it) for the oracle check
    groups = p0 // 4 + np.arange(16) * (n // 4 // 16)
    rows = (groups[:, None] * 4 + np.arange(4)).reshape(-1)
    th = t.cpu().numpy()
    dh = d[torch.as_tensor(rows, device=dev)].cpu().numpy().view(np.complex128).reshape(64, N)
    fh = fc[torch.as_tensor(groups, device=dev)].cpu().numpy().view(np.complex128).reshape(16, N)
    del d, fc, fcop, fo
    torch.cuda.empty_cache()

    # --- rank 3 as bench.py runs it: the shard generated on its own device ---------------
    ds = torch.empty((n, N, 2), dtype=torch.float64, device=dev)
    fs = torch.empty((n // 4, N, 2), dtype=torch.float64, device=dev)
    fos = torch.empty(n, dtype=torch.int32, device=dev)
    ts = torch.empty(N, dtype=torch.float64, device=dev)
    gpu._lib.check(L.gpd_synth_fill_dev(N, n, p0, SEED, 0.0, 0.002, 0.1, 0, gpu.M_2PI,
                                        ts.data_ptr(), ds.data_ptr(), N, fs.data_ptr(), N,
                                        fos.data_ptr(), None, 0, sptr))
    rank = fit(n, ts, ds.data_ptr(), fs.data_ptr(), n // 4, fos)
    assert rank.tobytes() == whole[p0:p1].tobytes(), "rank shard: records differ from the batch"
    # the generated shard is the batch's data for those series
    assert np.array_equal(ts.cpu().numpy(), th)
    loc = torch.as_tensor(rows - p0, device=dev)
    assert np.array_equal(ds[loc].cpu().numpy().view(np.complex128).reshape(64, N), dh)
    del ds, fs, fos, ts
    torch.cuda.empty_cache()

    # --- oracle spot check of the shard's records (harmonic evaluator, tie rule) --------
    fo_h = np.repeat(np.arange(16, dtype=np.int32), 4)
    ref = oracle.fit_batch(th, dh, fh, fo_h, flags=oracle.RECENTER)
    pert = [oracle.fit_batch(th, dh, fh, fo_h, flags=oracle.RECENTER, perturb_seed=s,
                             perturb_ulps=HARM_ULPS) for s in range(1, 13)]
    got = whole[rows]
    print(assert_fit_parity(got, ref, pert, label=f"C4 rank {RANK}/{WORLD}, 64 series x 1e5",
                            min_match=0.7))
