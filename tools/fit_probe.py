#!/usr/bin/env python3
"""Harmonic-fit probe (GPU box): device-resident synthetic batches (C3 generator, N samples) of
several sizes P; for each (P, series per wave) the k_fit_harmonic HIP-event time (median of
`reps` calls) and the records' hash (they must not depend on the setting).  With --prof, one
more call per setting with option fit_prof = 1: the library prints its cycle split on stderr
(the diagnostics build, GPD_LIB=diag or a --variant build with -DGPD_DIAG, adds NEWUOA's
phases).  One JSON line per setting."""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pixels", default="32,4096,12500")
    ap.add_argument("--lanes", default="0", help="option fit_lanes values (0 = automatic)")
    ap.add_argument("--lps", default="0", help="option fit_lps values (0 = automatic)")
    ap.add_argument("--wpb", default="0", help="option fit_wpb values (0 = automatic)")
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--prof", action="store_true")
    ap.add_argument("--offset", type=int, default=0, help="first series id (C4 rank shards)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import gpdemod_loader

    gpd = gpdemod_loader.load()
    L = gpd.load()
    applied = gpd.options_from_env()
    dev = torch.device("cuda", 0)
    sptr = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    err = ctypes.create_string_buffer(512)
    N = args.samples
    for P in [int(x) for x in args.pixels.split(",")]:
        G = (P + 3) // 4
        t = torch.empty(N, dtype=torch.float64, device=dev)
        d = torch.empty((P, N, 2), dtype=torch.float64, device=dev)
        fc = torch.empty((G, N, 2), dtype=torch.float64, device=dev)
        fcop = torch.empty(P, dtype=torch.int32, device=dev)
        gpd._lib.check(L.gpd_synth_fill_dev(N, P, args.offset, 7, 0.0, 0.002, 0.1, 0, gpd.M_2PI,
                                            t.data_ptr(), d.data_ptr(), N, fc.data_ptr(), N,
                                            fcop.data_ptr(), None, 0, sptr))
        out = torch.empty((P, 64), dtype=torch.uint8, device=dev)

        def call():
            gpd._lib.check(L.gpd_fit_batch_dev(N, P, t.data_ptr(), d.data_ptr(), N, fc.data_ptr(),
                                               G, N, fcop.data_ptr(), None, gpd.M_2PI, None,
                                               gpd.GPD_RECENTER, 60, out.data_ptr(), None, N, 0,
                                               sptr, err, len(err)), err)
        import itertools
        for lps, lanes, wpb in itertools.product(*[[int(x) for x in a.split(",")]
                                                   for a in (args.lps, args.lanes, args.wpb)]):
            gpd.set_option("fit_lps", lps)
            gpd.set_option("fit_lanes", lanes)
            gpd.set_option("fit_wpb", wpb)
            ks = {}
            for r in range(args.reps + 2):
                call()
                torch.cuda.synchronize(dev)
                if r >= 2:
                    for k, v in gpd.timings(0).items():
                        ks.setdefault(k, []).append(v)
            rec = out.cpu().numpy().tobytes()
            line = {"P": P, "fit_lps": lps, "fit_lanes": lanes, "fit_wpb": wpb, "options": applied,
                    "kernels_ms": {k: round(float(np.median(v)), 4) for k, v in ks.items()},
                    "records_sha": hashlib.sha256(rec).hexdigest()[:16]}
            print(json.dumps(line), flush=True)
            if args.prof:
                gpd.set_option("fit_prof", 1)
                print(f"--- prof P={P} lps={lps} fit_lanes={lanes} wpb={wpb}", file=sys.stderr,
                      flush=True)
                call()
                torch.cuda.synchronize(dev)
                gpd.set_option("fit_prof", 0)
        gpd.reset_options()
        gpd.options_from_env()
        del t, d, fc, fcop, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
