#!/usr/bin/env python3
"""Series per wave of the harmonic fit (option fit_lanes) against the batch size (GPU box): for each
P, device-resident synthetic series (N = 1e5, C3 generator), the fit kernel's HIP-event time per
lanes-per-wave setting, and the records of every setting compared byte for byte with the first setting's.
One JSON line per (P, lanes)."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pixels", default="32,128,256,512,1024,2048,4096,12500")
    ap.add_argument("--lanes", default="auto,64,32,16,8,4,2,1",
                    help="'auto': the library's own choice (fit_lanes_for, option fit_lanes = 0)")
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    import torch

    import gpdemod_loader

    gpd = gpdemod_loader.load()
    L = gpd.load()
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
        gpd._lib.check(L.gpd_synth_fill_dev(N, P, 0, 7, 0.0, 0.002, 0.1, 0, gpd.M_2PI, t.data_ptr(),
                                            d.data_ptr(), N, fc.data_ptr(), N, fcop.data_ptr(),
                                            None, 0, sptr))
        out = torch.empty((P, 64), dtype=torch.uint8, device=dev)
        ref = None
        for lanes in args.lanes.split(","):
            if lanes == "auto":
                gpd.set_option("fit_lanes", 0)
            else:
                gpd.set_option("fit_lanes", int(lanes))
            fit, step = [], []
            for r in range(args.reps + 2):
                s0 = torch.cuda.Event(enable_timing=True)
                s1 = torch.cuda.Event(enable_timing=True)
                s0.record()
                gpd._lib.check(L.gpd_fit_batch_dev(N, P, t.data_ptr(), d.data_ptr(), N, fc.data_ptr(),
                                                   G, N, fcop.data_ptr(), None, gpd.M_2PI, None,
                                                   gpd.GPD_RECENTER, 60, out.data_ptr(), None, N, 0,
                                                   sptr, err, len(err)), err)
                s1.record()
                torch.cuda.synchronize(dev)
                if r >= 2:
                    fit.append(gpd.timings(0).get("fit_harmonic", float("nan")))
                    step.append(s0.elapsed_time(s1))
            rec = out.cpu().numpy().tobytes()
            if ref is None:
                ref = rec
            print(json.dumps({"P": P, "lanes": lanes,
                              "waves": None if lanes == "auto" else -(-P // int(lanes)),
                              "fit_ms": round(float(np.median(fit)), 4),
                              "step_ms": round(float(np.median(step)), 4),
                              "records_equal_first": rec == ref}), flush=True)
        del t, d, fc, fcop, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
