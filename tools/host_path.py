#!/usr/bin/env python3
"""Host-buffer boundary timing (the Julia drop-in hands over host arrays: gpd_fit_batch).

0. C1, one diode × 1e4 samples (BASELINE configs[0]) against the oracle on one thread.
1. C2, one GRAVITY exposure (32 diodes + 8 FC columns × 1e5 samples, seed 42): wall time of
   the C-ABI call with the demodulated output (what demodulateall does), against the CPU
   oracle on the same exposure (16 OpenMP threads).
2. A larger host batch (P series × 1e5, generated on the device and copied to pageable host
   memory first): PCIe-inclusive throughput of gpd_fit_batch, fit only and with output.
Prints one JSON object.  Usage: python tools/host_path.py [--pixels P] [--reps R]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libgpdemod, as in tests/conftest.py)

import gpdemod_loader  # noqa: E402
import synth  # noqa: E402


def timed(fn, reps):
    fn()  # warm-up (workspace, module load)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pixels", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=16)
    a = ap.parse_args()
    gpd = gpdemod_loader.load()
    res = {}

    # ---- 0. C1: one diode × 1e4 samples (BASELINE configs[0]) ---------------------------------
    import oracle  # checker / CPU baseline only
    B1 = synth.make_batch(10_000, 1, seed=1)
    a1 = (B1["t"], B1["d"], B1["fc"], B1["fc_of_pixel"])
    s1, p1 = timed(lambda: gpd.fit_batch(*a1), a.reps)
    t0 = time.perf_counter()
    r1 = oracle.fit_batch(*a1, flags=oracle.RECENTER, nthreads=1)
    c1 = time.perf_counter() - t0
    res["C1"] = {"series": 1, "samples": 10_000, "host_call_ms": 1e3 * s1,
                 "device_kernels_ms": {k: round(v, 3) for k, v in gpd.timings(0).items()},
                 "cpu_oracle_ms_1_thread": 1e3 * c1,
                 "b": float(p1["b"][0]), "b_oracle": float(r1["b"][0]),
                 "b_truth": float(B1["truth"]["b"][0])}

    # ---- 1. C2: one exposure through the host boundary ------------------------------------
    B = synth.make_batch(a.samples, 32, seed=42)
    args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
    s_fit, _ = timed(lambda: gpd.fit_batch(*args), a.reps)
    s_out, (par, _) = timed(lambda: gpd.fit_batch(*args, want_output=True), a.reps)
    dev = gpd.timings(0)
    t0 = time.perf_counter()
    ref = oracle.fit_batch(*args, flags=oracle.RECENTER, nthreads=a.cpu_threads)
    s_cpu = time.perf_counter() - t0
    res["C2"] = {"series": 32, "samples": a.samples,
                 "host_call_ms_fit": 1e3 * s_fit, "host_call_ms_with_output": 1e3 * s_out,
                 "device_kernels_ms": {k: round(v, 3) for k, v in dev.items()},
                 "cpu_oracle_ms": 1e3 * s_cpu, "cpu_threads": a.cpu_threads,
                 "b_within_1e-10": int(np.sum(np.abs(par["b"] - ref["b"]) <= 1e-10 * np.abs(ref["b"])))}

    # ---- 2. larger host batch: PCIe-inclusive rate -----------------------------------------
    P, N = a.pixels - a.pixels % 4, a.samples
    L = gpd.load()
    dv = torch.device("cuda", 0)
    t = torch.empty(N, dtype=torch.float64, device=dv)
    d = torch.empty((P, N, 2), dtype=torch.float64, device=dv)
    fc = torch.empty((P // 4, N, 2), dtype=torch.float64, device=dv)
    fcop = torch.empty(P, dtype=torch.int32, device=dv)
    truth = torch.empty((P, 64), dtype=torch.uint8, device=dv)
    s = torch.cuda.current_stream(dv)
    rc = L.gpd_synth_fill_dev(N, P, 0, 7, 0.0, 0.002, 0.1, 0, gpd.M_2PI, t.data_ptr(),
                              d.data_ptr(), N, fc.data_ptr(), N, fcop.data_ptr(),
                              truth.data_ptr(), 0, ctypes.c_void_p(s.cuda_stream))
    gpd._lib.check(rc)
    torch.cuda.synchronize(dv)
    th = t.cpu().numpy()
    dh = d.cpu().numpy().view(np.complex128).reshape(P, N)
    fh = fc.cpu().numpy().view(np.complex128).reshape(P // 4, N)
    oh = fcop.cpu().numpy()
    del d, fc
    torch.cuda.empty_cache()
    b_fit, _ = timed(lambda: gpd.fit_batch(th, dh, fh, oh), max(2, a.reps // 2))
    dev_fit = gpd.timings(0)
    b_out, _ = timed(lambda: gpd.fit_batch(th, dh, fh, oh, want_output=True), max(2, a.reps // 2))
    # the same C-ABI call writing into an already-touched output array (Julia's demodulateall
    # writes into `output = copy(data)`; a fresh numpy array pays first-touch page faults)
    out = np.empty((P, N), dtype=np.complex128)
    out.fill(0)
    par = np.zeros(P, dtype=gpd.PARAM_DTYPE)
    err = ctypes.create_string_buffer(512)
    oh32 = np.ascontiguousarray(oh, dtype=np.int32)

    def call_touched():
        rc = L.gpd_fit_batch(N, P, gpd._lib.ptr(th), gpd._lib.ptr(dh), N, gpd._lib.ptr(fh), P // 4,
                             N, gpd._lib.ptr(oh32), None, float(gpd.M_2PI), None,
                             gpd.GPD_RECENTER, 60, gpd._lib.ptr(par), gpd._lib.ptr(out), N, 1,
                             err, len(err))
        gpd._lib.check(rc, err)

    b_touch, _ = timed(call_touched, max(2, a.reps // 2))
    nbytes = dh.nbytes + fh.nbytes + th.nbytes
    res["host_batch"] = {"series": P, "samples": N, "host_bytes_in": nbytes,
                         "fit_ms": 1e3 * b_fit, "fit_samples_per_s": P * N / b_fit,
                         "with_output_ms": 1e3 * b_out,
                         "with_output_samples_per_s": P * N / b_out,
                         "with_output_touched_ms": 1e3 * b_touch,
                         "with_output_touched_samples_per_s": P * N / b_touch,
                         "device_kernels_ms": {k: round(v, 3) for k, v in dev_fit.items()},
                         "host_memory": "pageable numpy arrays"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
