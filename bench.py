#!/usr/bin/env python3
"""Throughput of the per-pixel demodulation fit on MI355X (BASELINE.json metric).

One step = one full `demodulateall`-equivalent fit (grid + NEWUOA + π-flip check + final χ²,
src/Modulation.jl:388-432) of every series of the batch, inputs resident in HBM, parameter
records gathered to rank 0 (RCCL) — the demodulated-output pass is not part of the C3 workload
(160 GB of output cannot coexist with the 200 GB input).

Default workload (N=1): C3 = 1e5 synthetic series × 1e5 samples, fp64 complex, generated on
device (seeded counter RNG).  Multi-GPU (BASELINE C4): one process per GPU
(torch.distributed.run), strong scaling — the one C3 batch is split into contiguous series
shards (shard.shard_range, whole FC groups; 12 500 series per GPU at N = 8), each rank fits its
shard with no data-path collective and the 64-B records are gathered to rank 0 (RCCL).  The
moment sums do not depend on the shard (fixed sample units), so the gathered
records equal the 1-GPU run's bit for bit.  `--scaling weak` keeps 1e5 series per rank instead.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "complex samples/sec through demodulate fit (fp64), 1/2/4/8 MI355X + CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# dense fp64 matrix peak: v_mfma_f64_16x16x4 keeps the pipe 64 cycles per 2048 FLOP (measured,
# SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA, profiles/r1b/sq_counters.json) = 32 FLOP/clk/SIMD
# × 1024 SIMDs × 2.4 GHz
MFMA_F64_PEAK_TFLOPS = 78.6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pixels", type=int, default=100_000,
                    help="series in the batch (strong scaling) or per GPU (weak)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--dump-records", default=None,
                    help="rank 0 writes the gathered records (.npy, PARAM_DTYPE) here")
    ap.add_argument("--no-f64", action="store_true",
                    help="skip the all-f64 moment-kernel (option mix = 0) comparison steps")
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--t0", type=float, default=0.0)
    ap.add_argument("--method", default="auto", choices=["auto", "exact", "harmonic"])
    ap.add_argument("--cpu-pixels", type=int, default=2048,
                    help="series in the CPU-oracle baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: the CPUs this process may run on (sched_getaffinity), capped by "
                         "OMP_NUM_THREADS when the pool sets it (the box's CPU share)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sustain", type=float, default=None,
                    help="seconds of repeated steps after the timed region (0: off; default 8 "
                         "for the 1e5 x 1e5 headline shape, 0 otherwise)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the C5 block (faint exposure: GPU step + CPU oracle sample)")
    ap.add_argument("--no-c5-sweep", action="store_true",
                    help="skip the C5 Float32 storage / arithmetic tolerance sweep")
    ap.add_argument("--c5-cpu-pixels", type=int, default=256,
                    help="series of the C5 exposure in its CPU-oracle sample")
    ap.add_argument("--no-ceiling", action="store_true",
                    help="skip the reference-ceiling oracle runs (alternative summation orders, "
                         "1-ulp χ²) of the C3 CPU sample")
    ap.add_argument("--no-c2", action="store_true",
                    help="skip the C2 block (one exposure through the host-buffer drop-in call)")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the C4-rank rehearsal block (profiling runs: one kernel shape)")
    ap.add_argument("--dist-always", action="store_true",
                    help="initialise torch.distributed even at world size 1 (launch with "
                         "torch.distributed.run --nproc-per-node 1) and send the records through "
                         "the gather and the time through all_reduce: the RCCL branch of an "
                         "8-GPU run, exercised on one GPU")
    ap.add_argument("--storage", default="c64", choices=["c64", "c32"],
                    help="c32: series/FC kept as ComplexF32 in HBM (FITS VOLT precision, "
                         "gpd_fit_batch_c32_dev; arithmetic stays fp64)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch

    import gpdemod_loader

    gpd = gpdemod_loader.load()
    L = gpd.load()
    from gpdemod import shard  # noqa: E402  (package loaded by path as `gpdemod`)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run")
    # GPD_DIST_BACKEND=gloo: rehearsal of the multi-rank path with several ranks on fewer GPUs
    # (ranks share devices round-robin, records gathered through host memory); the scaling runs
    # use the default "nccl" = RCCL over xGMI, one rank per GPU
    backend = os.environ.get("GPD_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    dist = None
    use_dist = world > 1 or args.dist_always
    if use_dist:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sptr = ctypes.c_void_p(stream.cuda_stream)

    N = args.samples
    P_total = args.pixels - args.pixels % 4
    if args.scaling == "strong":
        p0, p1 = shard.shard_range(P_total, world, rank)
        counts = shard.shard_counts(P_total, world)
    else:
        P_total *= world
        p0 = shard.weak_offset(P_total // world, rank)
        p1 = p0 + P_total // world
        counts = [P_total // world] * world
    P = p1 - p0
    G = P // 4
    offset = p0
    # --- device-resident synthetic batch (untimed setup) -----------------------------------
    c32 = args.storage == "c32"
    t = torch.empty(N, dtype=torch.float64, device=dev)
    fcop = torch.empty(P, dtype=torch.int32, device=dev)
    truth = torch.empty((P, 64), dtype=torch.uint8, device=dev)
    params = torch.empty((P, 64), dtype=torch.uint8, device=dev)
    if not c32:
        d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
        fc = torch.empty((G, N, 2), dtype=torch.float64, device=dev)
        rc = L.gpd_synth_fill_dev(N, P, offset, args.seed, args.t0, 0.002, 0.1, 0, gpd.M_2PI,
                                  t.data_ptr(), d.data_ptr(), N, fc.data_ptr(), N,
                                  fcop.data_ptr(), truth.data_ptr(), local, sptr)
        gpd._lib.check(rc)
    else:
        # the same series generated in Float64 blocks of whole FC groups, rounded to ComplexF32
        d = torch.empty((P, N, 2), dtype=torch.float32, device=dev)
        fc = torch.empty((G, N, 2), dtype=torch.float32, device=dev)
        blk = min(P, 8192)
        d64 = torch.empty((blk, N, 2), dtype=torch.float64, device=dev)
        f64 = torch.empty((blk // 4, N, 2), dtype=torch.float64, device=dev)
        for c0 in range(0, P, blk):
            nb = min(blk, P - c0)
            rc = L.gpd_synth_fill_dev(N, nb, offset + c0, args.seed, args.t0, 0.002, 0.1, 0,
                                      gpd.M_2PI, t.data_ptr(), d64.data_ptr(), N, f64.data_ptr(),
                                      N, fcop[c0:].data_ptr(), truth[c0:].data_ptr(), local, sptr)
            gpd._lib.check(rc)
            d[c0:c0 + nb].copy_(d64[:nb])
            fc[c0 // 4:(c0 + nb) // 4].copy_(f64[:nb // 4])
        del d64, f64
        fcop.copy_(torch.arange(P, device=dev, dtype=torch.int32) // 4)
    torch.cuda.synchronize(dev)

    flags = gpd.GPD_RECENTER | {"auto": 0, "exact": gpd.GPD_METHOD_EXACT,
                                "harmonic": gpd.GPD_METHOD_HARMONIC}[args.method]
    err = ctypes.create_string_buffer(512)

    fit_dev = L.gpd_fit_batch_c32_dev if c32 else L.gpd_fit_batch_dev
    # per-step time of the record gather on this rank (ms): HIP events on the launch stream
    # around the RCCL gather (the current stream waits for the collective), host clock around
    # the gloo gather (after the records' device-to-host copy, which waits for the fit)
    gather_ms = []

    def step(timed=False):
        r = fit_dev(N, P, t.data_ptr(), d.data_ptr(), N, fc.data_ptr(), G, N,
                    fcop.data_ptr(), None, gpd.M_2PI, None, flags, 60,
                    params.data_ptr(), None, N, local, sptr, err, len(err))
        gpd._lib.check(r, err)
        if backend != "nccl" and use_dist:
            host = params.cpu()
            tg = time.perf_counter()
            g = shard.gather_records(host, world, rank, counts=counts, force=use_dist)
            if timed:
                gather_ms.append(1e3 * (time.perf_counter() - tg))
            return None if g is None else g.to(dev)
        if timed and use_dist:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        g = shard.gather_records(params, world, rank, counts=counts, force=use_dist)
        if timed and use_dist:
            e1.record(stream)
            gather_ms.append((e0, e1))
        return g

    log = (lambda msg: print(f"[bench] rank {rank}: {msg}", file=sys.stderr, flush=True))
    log(f"{P} series x {N} samples resident; {args.warmup} warmup + {args.steps} timed steps")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kern = {}
    t_start = time.perf_counter()
    for _ in range(args.steps):
        gathered = step(timed=True)
        for name, ms in gpd.timings(local).items():  # HIP events on the launch stream
            kern.setdefault(name, []).append(ms)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    own_elapsed = elapsed
    if dist:
        e = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    # every rank's own numbers, gathered to all (untimed): a shortfall from linear scaling then
    # shows whether it came from shard imbalance, a slow kernel on one GPU or the gather
    ranks = None
    if dist:
        g_ms = [x if isinstance(x, float) else x[0].elapsed_time(x[1]) for x in gather_ms]
        mine = {"rank": rank, "local_rank": local, "device": torch.cuda.get_device_name(dev),
                "series": P, "series_range": [p0, p1],
                "step_ms": round(1e3 * own_elapsed / args.steps, 3),
                "gather_ms": round(float(np.mean(g_ms)), 3) if g_ms else None,
                "kernels_ms": {k: round(float(np.mean(v)), 3) for k, v in kern.items()}}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)

    samples_total = float(P_total) * N * args.steps
    value = samples_total / elapsed
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    if args.dump_records:
        recs = (gathered if use_dist else params).cpu().numpy().reshape(-1).view(gpd.PARAM_DTYPE)
        np.save(args.dump_records, recs)

    # --- roofline of the dominant kernel (harmonic moment pass) ---------------------------
    rec = gpd.PARAM_DTYPE
    par = params.cpu().numpy().reshape(-1).view(rec)  # rank 0's shard
    roofline = None
    esz = 8 if c32 else 16  # stored bytes per complex sample
    algo_bytes = P * N * (esz + esz / 4) + 8 * N  # d + FC shared by 4 + t
    mom = kern.get("moments")
    if mom:
        avg_ms = float(np.mean(mom))
        achieved = algo_bytes / (avg_ms * 1e-3) / 1e9
        # the same kernel against the dense fp64 MFMA peak: 4 real MACs per harmonic per
        # complex sample for the harmonics 1..16 on the f64 MFMAs (17..24 run on split-bf16
        # MFMAs; option mix = 0: all 24 on f64)
        n_f64 = 24 if gpd.get_option("mix") == 0 else 16
        mfma_flops = 2.0 * 4 * n_f64 * P * N
        tflops = mfma_flops / (avg_ms * 1e-3) / 1e12
        roofline = {"bound": "hbm", "kernel": "k_moments", "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic_from_profiles(P, N, args.storage),
                    "traffic_source": "committed rocprofv3 PMC summary of this shape "
                                      "(profiles/pmc_moments*.json: FETCH_SIZE x2 + WRITE_SIZE per "
                                      "launch), not measured in this run",
                    "algorithmic_bytes": algo_bytes,
                    "avg_ms": round(avg_ms, 3),
                    "mfma": {"achieved": round(tflops, 2), "peak": MFMA_F64_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": round(tflops / MFMA_F64_PEAK_TFLOPS, 4),
                             "algorithmic_flops": mfma_flops,
                             "harmonics_f64": n_f64, "harmonics_bf16x3": 24 - n_f64}}
    kernels = {k: round(float(np.mean(v)), 3) for k, v in kern.items()}
    status = par["status"]
    fits = {"fallback_exact": int(np.count_nonzero(status & gpd.GPD_ST_FALLBACK)),
            "maxfun": int(np.count_nonzero(status & gpd.GPD_ST_MAXFUN)),
            "nan": int(np.count_nonzero(status & gpd.GPD_ST_NAN)),
            "mean_nfev": round(float(par["nfev"].mean()), 2)}
    tr = truth.cpu().numpy().reshape(-1).view(rec)
    fits["median_abs_b_err_vs_truth"] = float(np.median(np.abs(par["b"] - tr["b"])))

    # the same steps with every harmonic on the f64 MFMAs (option mix = 0; the production kernel puts
    # harmonics 17..24 on split-bf16 MFMAs), untimed by the headline
    f64_all = None
    if not args.no_f64 and world == 1:
        log("all-f64 moment kernel comparison steps (option mix = 0)")
        gpd.set_option("mix", 0)
        try:
            step()
            torch.cuda.synchronize(dev)
            km = []
            t1 = time.perf_counter()
            for _ in range(args.steps):
                step()
                km.append(gpd.timings(local).get("moments", float("nan")))
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t1
        finally:
            gpd.set_option("mix", 1)
        par64 = params.cpu().numpy().reshape(-1).view(rec).copy()
        step()  # leave the production records in `params`
        torch.cuda.synchronize(dev)
        f64_all = {"value": float(P_total) * N * args.steps / el,
                   "ms_per_step": 1e3 * el / args.steps,
                   "moments_ms": round(float(np.mean(km)), 3),
                   "note": "option mix = 0: all 24 harmonics on v_mfma_f64_16x16x4 (not the headline)",
                   "records": par64}

    # one C4 rank rehearsed on this GPU: the shard an 8-GPU node's rank fits (12 500 series of
    # the resident batch, a view — its records equal the batch's bit for bit, tests/test_gpu_c4.py),
    # timed the same way; the driver measures the 8-GPU run itself
    c4 = None
    if (world == 1 and (P_total, N) == (100_000, 100_000) and args.scaling == "strong"
            and not args.no_c4):
        n8 = shard.shard_counts(P_total, 8)[0]
        fo8 = fcop[:n8].contiguous()
        p8 = torch.empty((n8, 64), dtype=torch.uint8, device=dev)

        def step8():
            r = fit_dev(N, n8, t.data_ptr(), d.data_ptr(), N, fc.data_ptr(), n8 // 4, N,
                        fo8.data_ptr(), None, gpd.M_2PI, None, flags, 60, p8.data_ptr(), None, N,
                        local, sptr, err, len(err))
            gpd._lib.check(r, err)
        for _ in range(2):
            step8()
        torch.cuda.synchronize(dev)
        k8 = {}
        t8 = time.perf_counter()
        for _ in range(args.steps):
            step8()
            for name, ms in gpd.timings(local).items():
                k8.setdefault(name, []).append(ms)
        torch.cuda.synchronize(dev)
        ms8 = 1e3 * (time.perf_counter() - t8) / args.steps
        c4 = {"series": n8, "ms_per_step": round(ms8, 3),
              "kernels_ms": {k: round(float(np.mean(v)), 3) for k, v in k8.items()},
              "projected_speedup_at_8_gpus": round(1e3 * elapsed / args.steps / ms8, 2),
              "note": "rank 0's shard of the C4 split fitted alone on this GPU (no gather); "
                      "not the measured 8-GPU scaling"}

    # sustained run: the same step repeated for ~args.sustain seconds after the timed region
    # (untimed by the headline), in chunks of 10 steps — the steady-state rate once the clock
    # has settled under continuous HBM streaming + fp64 MFMA load (DVFS)
    sustained = None
    sustain = args.sustain if args.sustain is not None else (
        8.0 if (P_total, N) == (100_000, 100_000) else 0.0)
    if world == 1 and sustain > 0:
        chunks, n_done, ts = [], 0, time.perf_counter()
        while time.perf_counter() - ts < sustain:
            tc = time.perf_counter()
            for _ in range(10):
                step()
            torch.cuda.synchronize(dev)
            chunks.append(1e3 * (time.perf_counter() - tc) / 10)
            n_done += 10
        sustained = {"steps": n_done, "seconds": round(time.perf_counter() - ts, 2),
                     "ms_per_step_mean": round(float(np.mean(chunks)), 3),
                     "ms_per_step_min": round(float(np.min(chunks)), 3),
                     "ms_per_step_max": round(float(np.max(chunks)), 3),
                     "value_mean": float(P_total) * N / (float(np.mean(chunks)) * 1e-3),
                     "note": "chunks of 10 steps after the timed region; not the headline"}

    # BASELINE configs[1] (C2): one exposure through the drop-in call as the reference makes it
    # (host arrays in, output = copy(data) back), PCIe included
    c2 = None
    if world == 1 and not args.no_c2 and P >= 32 and not c32:
        c2 = c2_block(gpd, t, d, fc, args, log)

    cpu = None
    if not args.no_cpu and args.cpu_pixels > 0 and world == 1:  # rank 0 at N=1 only
        cpu = cpu_baseline(gpd, t, d, fc, fcop, par, args, N,
                           par64=None if f64_all is None else f64_all["records"])
    if f64_all is not None:
        del f64_all["records"]

    # BASELINE configs[4] (C5): one faint exposure, GPU step + CPU oracle sample (after the C3
    # batch is released: the exposure needs 8 GB more)
    c5 = None
    if (world == 1 and not args.no_c5 and (P_total, N) == (100_000, 100_000)
            and args.scaling == "strong"):
        del d, fc
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        c5 = c5_block(gpd, L, dev, sptr, args, log)

    out = {
        "metric": METRIC, "value": value, "unit": "complex samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (device-generated, seeded counter RNG; SURVEY §8d model)",
        "config": {"workload": ("C3" if world == 1 else "C4") if (P_total, N) == (100_000, 100_000)
                   else f"{P_total}x{N}",
                   "series_per_gpu": P, "samples": N, "total_series": P_total,
                   "method": args.method, "t0": args.t0, "storage": args.storage,
                   "parallelism": f"series-shard x{world}",
                   "gather": ("none" if not use_dist else "RCCL gather of 64-B records to rank 0"
                              if backend == "nccl" else f"{backend} gather (multi-rank rehearsal)")},
        "roofline": roofline, "cpu_baseline": cpu, "kernels_ms": kernels, "fits": fits,
        "all_f64_moments": f64_all, "c4_rank_rehearsal": c4, "sustained": sustained,
        "c2_exposure": c2,
        "c5_faint": c5,
        "distributed": None if not dist else {
            "world_size": dist.get_world_size(), "backend": backend,
            "per_rank": ranks,
            "step_ms_max_over_min": round(max(r["step_ms"] for r in ranks) /
                                          max(1e-9, min(r["step_ms"] for r in ranks)), 4),
            "note": "per rank: its own timed-loop time per step (before the MAX over ranks), "
                    "its kernels (HIP events, mean of the timed steps) and its record gather "
                    "(events around the RCCL gather on the launch stream; host clock for gloo)"},
        "build_id": gpd.build_id(),
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


def c2_block(gpd, t, d, fc, args, log, reps=5):
    """BASELINE configs[1] (C2): one GRAVITY exposure — 32 diodes + 8 FC columns x N samples, the
    first 32 series and 8 FC columns of the resident batch — through the drop-in boundary as the
    reference is called (src/GPPupilDemodulation.jl:161,205 → demodulateall, src/Modulation.jl:
    344-435): host arrays in, the demodulated `output = copy(data)` and the records back, PCIe
    included (gpd_fit_batch / gpd_fit_windows from pageable host memory).  `data` is the N x 40
    column-major matrix a Julia caller hands over (np.asfortranarray).  Median of `reps` calls
    each: the fit alone (records only), demodulateall with its output, demodulateall with
    fitoffsets (the reference's --center fit: the exact evaluator), and the 1-s windows of
    processmetrology (500 samples, gpd_fit_windows with the output)."""
    import numpy as np
    import torch

    N = t.shape[0]
    log(f"C2 exposure: 32 x {N} through the host-buffer drop-in ({reps} calls per case)")
    th = t.cpu().numpy()
    dd = d[:32].cpu().numpy().view(np.complex128).reshape(32, N)
    ff = fc[:8].cpu().numpy().view(np.complex128).reshape(8, N)
    data = np.empty((N, 40), dtype=np.complex128, order="F")
    fop = np.array([gpd.fc_column_of(c) - 1 for c in range(1, 33)], dtype=np.int32)
    for c in range(32):
        data[:, c] = dd[c]
    for g in range(8):  # diodes 4g..4g+3 share FC row g (the synthetic batch's groups of 4)
        data[:, fop[4 * g]] = ff[g]
    cols = data.T  # (40, N) C-contiguous view: no copy

    def med(fn):
        fn()
        ts = []
        for _ in range(reps):
            t1 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t1)
        return round(1e3 * float(np.median(ts)), 3), gpd.timings(0)

    # demodulateall returns a fresh N x 40 output per call (as the reference does): its pages
    # are faulted inside the call; the previous result's release (numpy unmapping 64 MB the
    # library's copy threads touched) is the caller's garbage collection, timed apart — each
    # call's result is kept until the timed calls are over
    def med_kept(fn):
        keep = [fn()]
        ts = []
        for _ in range(reps):
            t1 = time.perf_counter()
            keep.append(fn())
            ts.append(time.perf_counter() - t1)
        n = len(keep)
        t1 = time.perf_counter()
        keep.clear()
        rel = (time.perf_counter() - t1) / n
        return round(1e3 * float(np.median(ts)), 3), gpd.timings(0), round(1e3 * rel, 3)

    cases = {}
    ms, k = med(lambda: gpd.fit_batch(th, cols[:32], cols, fop))
    cases["fit_only"] = {"host_call_ms": ms, "what": "gpd_fit_batch, records only"}
    kern = k
    ms, k, rel = med_kept(lambda: gpd.demodulateall(th, data))
    cases["demodulateall"] = {"host_call_ms": ms, "release_of_the_output_ms": rel,
                              "what": "output = copy(data) with the 32 demodulated columns "
                                      "written in place, records, likelihood (a fresh output "
                                      "per call; its release by the caller timed apart); "
                                      "pageable data: one part (option h2d_parts automatic)"}
    # the same exposure in page-locked host memory (a caller that pins its buffers once): the
    # library then cuts the call into 2 parts, part 1's H2D DMA'd under part 0's kernels and
    # part 0's output back meanwhile (option h2d_parts automatic); and with h2d_parts = 1
    pin = torch.empty((40, N), dtype=torch.complex128, pin_memory=True).numpy()
    pin[:] = cols
    pdata = pin.T  # N x 40, column-major, page-locked
    ms, k, rel = med_kept(lambda: gpd.demodulateall(th, pdata))
    cases["demodulateall_pinned_input"] = {"host_call_ms": ms, "release_of_the_output_ms": rel,
                                           "h2d_parts": 2}
    parts = gpd.get_option("h2d_parts")
    gpd.set_option("h2d_parts", 1)
    try:
        ms, k, rel = med_kept(lambda: gpd.demodulateall(th, pdata))
        cases["demodulateall_pinned_input_one_part"] = {"host_call_ms": ms,
                                                        "release_of_the_output_ms": rel}
    finally:
        gpd.set_option("h2d_parts", parts)
    _, par_p, _ = gpd.demodulateall(th, pdata)
    same_pinned = [(p.a, p.b, p.ϕ) for p in par_p] == [(p.a, p.b, p.ϕ) for p in gpd.demodulateall(th, data)[1]]
    ms, k, rel = med_kept(lambda: gpd.demodulateall(th, data, fitoffsets=True))
    cases["demodulateall_fitoffsets"] = {
        "host_call_ms": ms, "release_of_the_output_ms": rel,
        "kernels_ms": {a: round(b, 3) for a, b in k.items()},
        "what": "--center fit (ModulationWithOffsets): the exact evaluator by default"}
    nwin = gpd.window_length(th, 1.0)
    out = cols.copy()

    def windows():
        gpd.fit_windows(th, cols[:32], cols, fop, nwin, want_output=True, out=out[:32])
    ms, k = med(windows)
    cases["windows_1s"] = {"host_call_ms": ms, "window_samples": nwin,
                           "series": 32 * (-(-N // nwin)),
                           "kernels_ms": {a: round(b, 3) for a, b in k.items()},
                           "what": "processmetrology's window mode: every 1-s window fitted "
                                   "(gpd_fit_windows), demodulated output in place"}
    # the same calls' records against the fit-only call: the output path changes nothing
    p_fit = gpd.fit_batch(th, cols[:32], cols, fop)
    _, par, _ = gpd.demodulateall(th, data)
    same = bool(np.array_equal(np.array([p.b for p in par]), p_fit["b"]))
    return {"series": 32, "samples": N, "fc_columns": 8,
            "host_bytes_in": int(dd.nbytes + ff.nbytes + th.nbytes),
            "host_bytes_out": int(dd.nbytes), "cases": cases,
            "kernels_ms_fit_only": {a: round(b, 3) for a, b in kern.items()},
            "records_equal_fit_only": same,
            "records_equal_pinned_two_parts": same_pinned,
            "host_memory": "pageable numpy arrays (column-major, as a Julia Matrix)",
            "note": "PCIe-inclusive host-buffer calls; not the headline (which is HBM-resident)"}


def c5_block(gpd, L, dev, sptr, args, log):
    """BASELINE configs[4] (C5): one faint exposure (tools/c5_sweep.py's workload: 4096 series ×
    1e5 samples, seed 11, HIGH/NORMAL/LOW states with TRANSIENT margins, power 1.1 : 0.1 : 0.01,
    Float64), resident in HBM.  GPU: the default (harmonic) faint fit, `args.steps` timed calls
    (HIP events per kernel).  CPU: the oracle on the first `c5_cpu_pixels` series at 8 threads
    (the reference's Threads.@threads width, src/Modulation.jl:387) and at the box's share, plus
    the parity of that sample (exact evaluator bit for bit; harmonic within 1e-10 or a NEWUOA tie)."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from c5_sweep import POWER, c5_states

    P, N = 4096, args.samples
    G = P // 4
    log(f"C5 faint exposure {P} x {N}")
    t = torch.empty(N, dtype=torch.float64, device=dev)
    d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
    fc = torch.empty((G, N, 2), dtype=torch.float64, device=dev)
    fcop = torch.empty(P, dtype=torch.int32, device=dev)
    gpd._lib.check(L.gpd_synth_fill_dev(N, P, 0, 11, 0.0, 0.002, 0.0, 0, gpd.M_2PI, t.data_ptr(),
                                        d.data_ptr(), N, fc.data_ptr(), N, fcop.data_ptr(), None,
                                        dev.index, sptr))
    th = t.cpu().numpy()
    st = c5_states(gpd, th)
    power = torch.tensor([POWER[int(x)] for x in st], dtype=torch.float64, device=dev)
    d.mul_(power[None, :, None])
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    d.add_(torch.randn(d.shape, dtype=torch.float64, device=dev, generator=gen),
           alpha=0.02 / np.sqrt(2.0))
    std = torch.from_numpy(st).to(dev)
    params = torch.empty((P, 64), dtype=torch.uint8, device=dev)
    err = ctypes.create_string_buffer(512)

    def call(method, dd=None, ff=None):
        c32 = dd is not None
        fn = L.gpd_fit_batch_c32_dev if c32 else L.gpd_fit_batch_dev
        dd, ff = (dd, ff) if c32 else (d, fc)
        gpd._lib.check(fn(N, P, t.data_ptr(), dd.data_ptr(), N, ff.data_ptr(), G,
                          N, fcop.data_ptr(), std.data_ptr(), gpd.M_2PI, None,
                          gpd.GPD_RECENTER | method, 60, params.data_ptr(),
                          None, N, dev.index, sptr, err, len(err)), err)

    for _ in range(2):
        call(0)
    torch.cuda.synchronize(dev)
    kern = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        call(0)
        for name, ms in gpd.timings(dev.index).items():
            kern.setdefault(name, []).append(ms)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    rec = gpd.PARAM_DTYPE
    par = params.cpu().numpy().reshape(-1).view(rec).copy()
    nvalid = int(np.count_nonzero((st != gpd.MetState.TRANSIENT)))
    ms = 1e3 * el / args.steps
    out = {"series": P, "samples": N, "valid_samples": nvalid,
           "gpu": {"ms_per_step": round(ms, 3), "complex_samples_per_s": P * N / (ms * 1e-3),
                   "valid_samples_per_s": P * nvalid / (ms * 1e-3),
                   "roofline_frac_20B": round(P * N * 20.0 / (ms * 1e-3) / 8e12, 4),
                   "kernels_ms": {k: round(float(np.mean(v)), 3) for k, v in kern.items()},
                   "method": "auto (harmonic, faint statistics fused into the moment pass)"}}
    # the exact evaluator on the whole exposure (the reference's arithmetic; the path of
    # --center fit and of the harmonic fallback): one warm and two timed calls
    call(gpd.GPD_METHOD_EXACT)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(2):
        call(gpd.GPD_METHOD_EXACT)
    torch.cuda.synchronize(dev)
    ems = 1e3 * (time.perf_counter() - t0) / 2
    out["gpu_exact"] = {"ms_per_step": round(ems, 2), "complex_samples_per_s": P * N / (ems * 1e-3),
                        "kernels_ms": {k: round(float(v), 3) for k, v in gpd.timings(dev.index).items()}}
    par_exact = params.cpu().numpy().reshape(-1).view(rec).copy()
    if not args.no_c5_sweep:
        sw = c5_fp32_sweep(gpd, call, params, d, fc, dev, P, N,
                           {"f64_harmonic": par, "f64_exact": par_exact}, log)
        sw["rows"]["f64_harmonic"] = {"ms": round(ms, 3)}
        sw["rows"]["f64_exact"] = {"ms": round(ems, 2)}
        sw["fp32_arith_speedup_over_f64_exact"] = round(ems / sw["rows"]["fp32"]["ms"], 3)
        out["fp32_sweep"] = sw
    if args.no_cpu or args.c5_cpu_pixels <= 0:
        return out
    # the sample: the first k series through the oracle, and the GPU's exact evaluator on them
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / CPU baseline only

    k = min(args.c5_cpu_pixels, P) // 4 * 4
    dd = d[:k].cpu().numpy().view(np.complex128).reshape(k, N)
    ff = fc[: k // 4].cpu().numpy().view(np.complex128).reshape(k // 4, N)
    fo = fcop[:k].cpu().numpy()
    threads, _ = cpu_threads(args.cpu_threads)
    runs = {}
    for nth in sorted({min(8, threads), threads}):
        t1 = time.perf_counter()
        ref = oracle.fit_batch(th, dd, ff, fo, state=st, flags=oracle.RECENTER, nthreads=nth)
        runs[nth] = time.perf_counter() - t1
    # GPU exact evaluator on the same sample (host-buffer call): the oracle's bits
    ex = gpd.fit_batch(th, dd, ff, fo, state=st, method="exact")
    exact_equal = all(np.array_equal(ex[f], ref[f]) for f in ("b", "phi", "chi2", "a", "nfev"))
    e = np.max([np.abs(par["b"][:k] - ref["b"]) / np.abs(ref["b"]),
                np.abs((par["phi"][:k] - ref["phi"] + np.pi) % (2 * np.pi) - np.pi),
                np.abs(par["a"][:k] - ref["a"]) / np.abs(ref["a"])], axis=0)
    out["cpu_baseline"] = {
        "kind": "port", "sample": f"first {k} series of the C5 exposure x {N} samples, "
                                  f"oracle/ C restatement (faint: compute_mean_var_power + "
                                  f"weighted fit), OpenMP over series",
        "seconds": {str(n): round(v, 3) for n, v in runs.items()},
        "complex_samples_per_s": {str(n): k * N / v for n, v in runs.items()},
        "cores": threads}
    out["parity_sample"] = {"series": k, "exact_evaluator_bitwise": bool(exact_equal),
                            "harmonic_within_1e-10": f"{int((e <= 1e-10).sum())}/{k}",
                            "harmonic_within_1e-6": f"{int((e <= 1e-6).sum())}/{k}",
                            "harmonic_max_dev": float(e.max())}
    return out


def c5_fp32_sweep(gpd, call, params, d, fc, dev, P, N, ref, log):
    """BASELINE configs[4]'s fp32-vs-fp64 tolerance sweep on the C5 exposure, on this build
    (verdict r5 item 3; tools/c5_sweep.py's pairs and summaries).  Rows, each against the Float64
    records of the same evaluator:
      c32_harmonic / c32_exact  ComplexF32 STORAGE (the FITS VOLT precision, d and FC rounded to
                                Float32 and kept so in HBM; Float64 arithmetic) — gpd_fit_batch_c32_dev
      fp32 / c32_fp32           Float32 ARITHMETIC (GPD_FP32: the exact evaluator's per-sample
                                θ, sin, sincos, phasor, model and residual in Float32; sums and
                                NEWUOA in Float64) on the Float64 and on the ComplexF32 data,
                                against the Float64 exact evaluator
    plus harmonic vs exact in Float64 (the scale of evaluator-level differences).  Columns: the
    fraction of series within 1e-3 … 1e-8 and the max, for b (relative), ϕ and arg a (radians),
    |a| (relative) and all four together; each row's time (one warm call, then one timed call,
    wall clock around the device call)."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from c5_sweep import summarise

    rec = gpd.PARAM_DTYPE
    d32, fc32 = d.float(), fc.float()
    rows = {}
    res = dict(ref)

    def timed(key, method, c32):
        args = (d32, fc32) if c32 else ()
        call(method, *args)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        call(method, *args)
        torch.cuda.synchronize(dev)
        ms = 1e3 * (time.perf_counter() - t0)
        res[key] = params.cpu().numpy().reshape(-1).view(rec).copy()
        rows[key] = {"ms": round(ms, 2),
                     "fallback": int(np.count_nonzero(res[key]["status"] & gpd.GPD_ST_FALLBACK)),
                     "nan": int(np.count_nonzero(res[key]["status"] & gpd.GPD_ST_NAN))}
        log(f"C5 sweep {key}: {ms:.1f} ms")

    timed("c32_harmonic", 0, True)
    timed("c32_exact", gpd.GPD_METHOD_EXACT, True)
    timed("fp32", gpd.GPD_FP32, False)
    timed("c32_fp32", gpd.GPD_FP32, True)
    del d32, fc32
    torch.cuda.empty_cache()
    pairs = {"c32_storage_harmonic_vs_f64_harmonic": ("c32_harmonic", "f64_harmonic"),
             "c32_storage_exact_vs_f64_exact": ("c32_exact", "f64_exact"),
             "fp32_arith_vs_f64_exact": ("fp32", "f64_exact"),
             "fp32_arith_c32_data_vs_f64_exact": ("c32_fp32", "f64_exact"),
             "f64_harmonic_vs_f64_exact": ("f64_harmonic", "f64_exact")}
    table = {}
    for name, (a, b) in pairs.items():
        s = summarise(res[a], res[b])
        table[name] = {"within": s["all_params"]["within"], "max": s["all_params"]["max"],
                       "per_param": {k: {"max": v["max"], "within": v["within"]}
                                     for k, v in s.items() if k != "all_params"}}
    return {"series": P, "samples": N, "rows": rows, "pairs": table,
            "note": "ComplexF32 storage = Float32 data, Float64 engine (both evaluators); "
                    "Float32 arithmetic = GPD_FP32 exact evaluator; deviations per series of b "
                    "(relative), ϕ / arg a (radians, mod 2π), |a| (relative)"}


def traffic_from_profiles(P, N, storage="c64"):
    """HBM bytes per moment-kernel launch from a committed rocprofv3 PMC summary
    (profiles/pmc_moments*.json: FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM + WRITE_SIZE),
    when one was taken on this shape and storage."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_moments*.json"))):
        try:
            with open(path) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        st = j.get("storage", "c32" if "c32" in os.path.basename(path) else "c64")
        if j.get("pixels") == P and j.get("samples") == N and st == storage:
            return j.get("hbm_bytes_per_launch")
    return None


def cpu_threads(requested=0):
    """Threads for the CPU baseline and what the box offers: the CPUs this process may run on
    (sched_getaffinity), capped by OMP_NUM_THREADS when the GPU pool sets it (the box's CPU
    share; nproc counts the whole machine)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    n = requested or aff
    if not requested and omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n), {"nproc": os.cpu_count(), "affinity": aff, "omp_num_threads": omp}


def cpu_baseline(gpd, t, d, fc, fcop, par, args, N, par64=None):
    """Oracle restatement (oracle/, C + OpenMP) on a bounded sample of the same device-resident
    series, timed on the host; also a full-size parity check of every series of the sample
    (harmonic evaluator: within 1e-10 or inside the oracle's own NEWUOA tie envelope)."""
    import shutil

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / CPU baseline only

    k = min(args.cpu_pixels, d.shape[0]) // 4 * 4
    th = t.cpu().numpy()
    # Float64.(data) of the stored series (c32 storage: the widened ComplexF32 values)
    dd = d[:k].double().cpu().numpy().view(np.complex128).reshape(k, N)
    ff = fc[: k // 4].double().cpu().numpy().view(np.complex128).reshape(k // 4, N)
    fo = fcop[:k].cpu().numpy()
    threads, machine = cpu_threads(args.cpu_threads)
    print(f"[bench] CPU baseline: oracle on {k} series x {N} samples, {threads} threads",
          file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    ref = oracle.fit_batch(th, dd, ff, fo, flags=oracle.RECENTER, nthreads=threads)
    dt = time.perf_counter() - t0

    # C2 (one exposure: 32 diodes sharing 8 FC columns) through the oracle, median of 3, with
    # the sample's thread count and with 8 threads — the reference's own width: its
    # Threads.@threads loop has 8 work items, (telescope, side) (src/Modulation.jl:387)
    def c2_runs(nth):
        runs = []
        for _ in range(3):
            t1 = time.perf_counter()
            oracle.fit_batch(th, dd[:32], ff[:8], fo[:32], flags=oracle.RECENTER, nthreads=nth)
            runs.append(time.perf_counter() - t1)
        return runs
    c2 = c2_runs(threads)
    c2_8 = c2_runs(min(8, threads)) if threads != 8 else c2

    def dev(x, r):
        dphi = np.abs((x["phi"] - r["phi"] + np.pi) % (2 * np.pi) - np.pi)
        return np.max([np.abs(x["b"] - r["b"]) / np.abs(r["b"]),
                       dphi / np.maximum(1.0, np.abs(r["phi"])),
                       np.abs(x["a"] - r["a"]) / np.abs(r["a"]),
                       np.abs(x["chi2"] - r["chi2"]) / np.abs(r["chi2"])], axis=0)

    pert_cache = {}  # perturbation seed -> {series: oracle record}

    def perturbed(seed, rows, ulps=128.0):
        """The oracle's fits of `rows` with χ² × (1 ± ulps·ulp) noise of `seed` (each series is
        fitted on its own; cached so the two parity checks share the runs)."""
        cache = pert_cache.setdefault((seed, ulps), {})
        need = np.array([r for r in rows if r not in cache], dtype=np.int64)
        if need.size:
            gsel = np.unique(fo[need])
            remap = {g: i for i, g in enumerate(gsel)}
            fo_s = np.array([remap[g] for g in fo[need]], dtype=np.int32)
            rec = oracle.fit_batch(th, dd[need], ff[gsel], fo_s, flags=oracle.RECENTER,
                                   nthreads=threads, perturb_seed=seed, perturb_ulps=ulps)
            for r, x in zip(need, rec):
                cache[int(r)] = x
        return np.array([cache[int(r)] for r in rows], dtype=ref.dtype)

    def tie_check(got, label):
        """Every series of the sample: within 1e-10 of the oracle, or an outcome the oracle itself
        reaches when its χ² moves by the harmonic evaluator's error size, or within 1.5× the
        spread of those outcomes, or — where the oracle itself re-routes in ≥ 1/4 of those runs —
        below NEWUOA's rhoend 1e-3 (tests/test_gpu_parity.assert_fit_parity).  Noise: 12 runs of
        χ² × (1 ± 128 ulp), the typical harmonic error; for series those leave unexplained, 36
        more at 512 ulp ≈ 1.1e-13, the harmonic χ² error bound (test_chi2_evaluation_parity).
        Perturbed runs only for series outside 1e-10."""
        e = dev(got, ref)
        out = {"within_1e-10": f"{int((e <= 1e-10).sum())}/{k}"}
        for lim in (1e-8, 1e-6, 1e-4, 1e-3):
            out[f"within_{lim:g}"] = f"{int((e <= lim).sum())}/{k}"
        out["max_dev"] = float(e.max())
        miss = np.nonzero(e > 1e-10)[0]
        unexplained = []
        if miss.size:
            print(f"[bench] {label}: {miss.size} series outside 1e-10, perturbed oracle runs",
                  file=sys.stderr, flush=True)
            g_m, r_m, e_m = got[miss], ref[miss], e[miss]

            def classify(pert):
                devs = np.array([dev(q, r_m) for q in pert])
                env = devs.max(axis=0)
                same = np.any([dev(g_m, q) <= 1e-10 for q in pert], axis=0)
                chaotic = (devs > 1e-10).mean(axis=0) >= 0.25
                return same, env, chaotic, same | (e_m <= 1.5 * env + 1e-10) | (chaotic & (e_m < 1e-3))

            pert = [perturbed(sd, miss) for sd in range(1, 13)]
            same, env, chaotic, explained = classify(pert)
            explained12 = explained.copy()  # by the 12 draws at 128 ulp alone
            nruns = np.full(miss.size, 12)
            if not explained.all():
                # the same rule with more draws of the oracle's χ² noise, for those series only
                sel = np.nonzero(~explained)[0]
                print(f"[bench] {label}: {sel.size} series need more draws",
                      file=sys.stderr, flush=True)
                more = [perturbed(sd, miss[sel], 512.0) for sd in range(13, 49)]
                sub_pert = [q[sel] for q in pert] + more
                devs = np.array([dev(q, r_m[sel]) for q in sub_pert])
                env_s = devs.max(axis=0)
                same_s = np.any([dev(g_m[sel], q) <= 1e-10 for q in sub_pert], axis=0)
                chaotic_s = (devs > 1e-10).mean(axis=0) >= 0.25
                same[sel], env[sel], chaotic[sel] = same_s, env_s, chaotic_s
                explained[sel] = same_s | (e_m[sel] <= 1.5 * env_s + 1e-10) | \
                    (chaotic_s & (e_m[sel] < 1e-3))
                nruns[sel] = 48
            unexplained = [int(i) for i in miss[~explained]]
            # how good a minimum the GPU's landing point is: the oracle's own χ² there against
            # the oracle's fitted χ² (a flat valley: both minima agree to ~rhoend²)
            dchi = []
            for i in miss:
                v, _ = oracle.chi2(th, dd[i], oracle.fc_phasor(ff[fo[i]]), got["b"][i],
                                   got["phi"][i])
                dchi.append((v - ref["chi2"][i]) / ref["chi2"][i])
            dchi = np.array(dchi)
            inside = ~same & (e_m <= 1.5 * env + 1e-10)
            out["outside_1e-10"] = {"n": int(miss.size),
                                    "perturbed_oracle_runs": {
                                        "12 at 128 ulp": int((nruns == 12).sum()),
                                        "12 at 128 + 36 at 512 ulp": int((nruns == 48).sum())},
                                    "oracle_chi2_at_gpu_point_rel": {
                                        "max": float(np.max(np.abs(dchi))),
                                        "median": float(np.median(dchi)),
                                        "lower_than_oracle_fit": int((dchi < 0).sum())},
                                    "equal_to_a_perturbed_oracle_outcome": int(same.sum()),
                                    "inside_1.5x_oracle_envelope": int(inside.sum()),
                                    "oracle_chaotic_below_rhoend": int((~same & ~inside & chaotic
                                                                        & (e_m < 1e-3)).sum())}
        out["unexplained"] = len(unexplained)
        out["unexplained_series"] = unexplained[:16]
        # the weaker explanations, reported beside `unexplained` (not folded into it): series
        # explained only after the 36 extra draws at 512 ulp, and series explained only by the
        # "oracle-chaotic, below rhoend" rule
        if miss.size:
            inside = same | (e_m <= 1.5 * env + 1e-10)
            out["explained_only_after_512ulp_draws"] = int((explained & ~explained12).sum())
            out["explained_only_by_chaotic_rule"] = int((explained & ~inside).sum())
        else:
            out["explained_only_after_512ulp_draws"] = 0
            out["explained_only_by_chaotic_rule"] = 0
        return out

    # C1 (BASELINE configs[0]): one diode x 1e4 samples, the oracle on one thread, median of 5;
    # the GPU's host-buffer call on the same diode beside it
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import synth

    B1 = synth.make_batch(10_000, 1, seed=42)
    a1 = (B1["t"], B1["d"], B1["fc"], B1["fc_of_pixel"])
    c1_cpu, c1_gpu = [], []
    for _ in range(5):
        t1 = time.perf_counter()
        r1 = oracle.fit_batch(*a1, flags=oracle.RECENTER, nthreads=1)
        c1_cpu.append(time.perf_counter() - t1)
    gpd.fit_batch(*a1)
    for _ in range(5):
        t1 = time.perf_counter()
        g1 = gpd.fit_batch(*a1, method="exact")
        c1_gpu.append(time.perf_counter() - t1)
    c1 = {"cpu_s_median_of_5": float(np.median(c1_cpu)), "cpu_runs": c1_cpu, "cpu_threads": 1,
          "gpu_host_call_s_median_of_5": float(np.median(c1_gpu)),
          "gpu_exact_equals_oracle": bool(all(np.array_equal(g1[f], r1[f])
                                              for f in ("b", "phi", "chi2", "a", "nfev"))),
          "what": "one diode x 1e4 samples (synthetic, seed 42): oracle fit on one thread; the "
                  "GPU's gpd_fit_batch on the host arrays (PCIe included), exact evaluator"}

    # the reference's own reproducibility at 1e-10: the oracle re-run on the same sample with
    # another legitimate summation order of the cost (Julia's @simd loops and BLAS zdotc fix none,
    # src/Modulation.jl:143-144,181,301 — 16 / 32 accumulators = an AVX2 / AVX-512 CPU) and with
    # χ² moved by one ulp; how many series each moves beyond 1e-10, and how many of the GPU's
    # series outside 1e-10 are series the reference itself does not reproduce at 1e-10
    ceiling = None
    if not args.no_ceiling:
        print("[bench] reference ceiling: oracle with other summation orders / 1-ulp chi2",
              file=sys.stderr, flush=True)
        variants = {"order_avx2_16acc": oracle.fit_batch(th, dd, ff, fo, flags=oracle.RECENTER,
                                                         nthreads=threads, order=16),
                    "order_avx512_32acc": oracle.fit_batch(th, dd, ff, fo, flags=oracle.RECENTER,
                                                           nthreads=threads, order=32),
                    "chi2_1ulp": oracle.fit_batch(th, dd, ff, fo, flags=oracle.RECENTER,
                                                  nthreads=threads, perturb_seed=1,
                                                  perturb_ulps=1.0)}
        gpu_out = dev(par[:k], ref) > 1e-10
        moved_any = np.zeros(k, bool)
        ceiling = {"what": "oracle re-runs of the C3 sample: CR8 (the product's order) vs other "
                           "orders a CPU may take, and vs chi2 x (1 +- 1 ulp); counts = series "
                           "moved beyond 1e-10 (any of b, phi, a, chi2)"}
        for name, v in variants.items():
            mv = dev(v, ref) > 1e-10
            moved_any |= mv
            ceiling[name] = {"moved_beyond_1e-10": f"{int(mv.sum())}/{k}",
                             "max_dev": float(dev(v, ref).max())}
        o16, o32 = variants["order_avx2_16acc"], variants["order_avx512_32acc"]
        ceiling["avx2_vs_avx512"] = {
            "moved_beyond_1e-10": f"{int((dev(o16, o32) > 1e-10).sum())}/{k}",
            "note": "the same reference arithmetic on two CPUs' summation orders"}
        ceiling["reference_not_reproducible_at_1e-10"] = f"{int(moved_any.sum())}/{k}"
        ceiling["gpu_outside_1e-10"] = int(gpu_out.sum())
        ceiling["gpu_outside_1e-10_on_series_the_reference_moves"] = int((gpu_out & moved_any).sum())
        near = np.min([dev(par[:k], v) for v in [ref, *variants.values()]], axis=0)
        ceiling["gpu_within_1e-10_of_some_reference_variant"] = f"{int((near <= 1e-10).sum())}/{k}"

    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(line.split(":", 1)[1].strip() for line in f
                             if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    res = {"value": k * N / dt, "unit": "complex samples/s", "cores": threads, "kind": "port",
           "value_per_core": k * N / dt / threads,
           "cpu_model": cpu_model, **machine,
           "julia": shutil.which("julia") or "not installed on this box (reference not runnable)",
           "sample": f"{k} of the device-generated series x {N} samples (first FC groups), "
                     f"oracle/ C restatement, OpenMP over series ({threads} threads), "
                     f"{dt:.1f} s wall",
           "c2_one_exposure_s": {"median_of_3": float(np.median(c2)), "runs": c2,
                                 "threads": threads,
                                 "median_of_3_at_8_threads": float(np.median(c2_8)),
                                 "runs_at_8_threads": c2_8,
                                 "samples_per_s_per_core_at_8_threads":
                                     32 * N / float(np.median(c2_8)) / min(8, threads),
                                 "what": "32 series x N samples (8 FC columns) through the "
                                         "oracle, the reference's per-exposure call; 8 threads "
                                         "= the width of its Threads.@threads loop "
                                         "(src/Modulation.jl:387)"},
           "c1_one_diode": c1,
           "parity": tie_check(par[:k], "harmonic (production moments)")}
    if ceiling is not None:
        res["parity"]["reference_ceiling"] = ceiling
    if par64 is not None:
        res["parity_all_f64_moments"] = tie_check(par64[:k], "harmonic (all-f64 moments)")
    return res


if __name__ == "__main__":
    main()
