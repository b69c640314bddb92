#!/usr/bin/env python3
"""Probe one C3 series the bench's tie check could not explain: GPU harmonic vs oracle fits,
χ² of each evaluator at both landing points, the cancellation factor κ = W2/(N χ²), the π-flip
status, and how large a χ² perturbation the oracle needs to land where the GPU does."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=1903)
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args()
    import numpy as np
    import torch

    import gpdemod_loader
    import oracle

    gpd = gpdemod_loader.load()
    L = gpd.load()
    dev = torch.device("cuda", 0)
    sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    N, P = args.samples, 4
    off = args.series // 4 * 4
    j = args.series - off
    t = torch.empty(N, dtype=torch.float64, device=dev)
    d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
    fc = torch.empty((1, N, 2), dtype=torch.float64, device=dev)
    fcop = torch.empty(P, dtype=torch.int32, device=dev)
    gpd._lib.check(L.gpd_synth_fill_dev(N, P, off, args.seed, 0.0, 0.002, 0.1, 0, gpd.M_2PI,
                                        t.data_ptr(), d.data_ptr(), N, fc.data_ptr(), N,
                                        fcop.data_ptr(), None, 0, sptr))
    torch.cuda.synchronize(dev)
    th = t.cpu().numpy()
    dd = d.cpu().numpy().view(np.complex128).reshape(P, N)
    ff = fc.cpu().numpy().view(np.complex128).reshape(1, N)
    fo = fcop.cpu().numpy() - fcop.cpu().numpy().min()
    harm = gpd.fit_batch(th, dd, ff, fo, method="harmonic")[j]
    exact = gpd.fit_batch(th, dd, ff, fo, method="exact")[j]
    ref = oracle.fit_batch(th, dd, ff, fo, flags=oracle.RECENTER)[j]
    p = oracle.fc_phasor(ff[0])
    out = {"series": args.series}
    for name, r in (("gpu_harmonic", harm), ("gpu_exact", exact), ("oracle", ref)):
        out[name] = {"b": float(r["b"]), "phi": float(r["phi"]), "chi2": float(r["chi2"]),
                     "nfev": int(r["nfev"]), "status": int(r["status"])}
        v, _ = oracle.chi2(th, dd[j], p, float(r["b"]), float(r["phi"]))
        out[name]["oracle_chi2_here"] = float(v)
        bp = np.tile([float(r["b"]), float(r["phi"])], (P, 1))
        out[name]["harmonic_chi2_here"] = float(
            gpd.chi2_batch(th, dd, ff, fo, bp, method="harmonic")["chi2"][j])
    W2 = float(np.sum(np.abs(dd[j]) ** 2))
    out["kappa_W2_over_N_chi2"] = W2 / (N * float(ref["chi2"]))
    reach = {}
    for ulps in (128, 512, 2048, 8192, 32768):
        hits = 0
        for sd in range(1, 25):
            q = oracle.fit_batch(th, dd, ff, fo, flags=oracle.RECENTER, perturb_seed=sd,
                                 perturb_ulps=float(ulps))[j]
            dv = max(abs(q["b"] - harm["b"]) / abs(harm["b"]), abs(q["phi"] - harm["phi"]))
            hits += dv <= 1e-10
        reach[str(ulps)] = int(hits)
    out["oracle_runs_landing_on_gpu_point_of_24"] = reach
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
