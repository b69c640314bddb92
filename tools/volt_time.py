#!/usr/bin/env python3
"""End-to-end exposure timing (GPU box): processmetrology's numeric core straight from a FITS-like
VOLT column (N rows × 80 Float32, 40 complex columns: 32 diodes + 8 FC), synthetic (synth seed 5,
Stefan centres of the reference's own data/Stefan_file.txt copied in tests/golden), through
process_volt — host Float32 rows in, demodulated Float32 rows out, PCIe included; the whole
exposure and 1-s windows, MJD-scale timestamps (TIME·1e-6 + 86400·MJD) or relative.  One JSON
line per case: median wall time of the call and the per-kernel HIP-event times."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (before libgpdemod)

    import gpdemod_loader
    import synth

    gpd = gpdemod_loader.load()
    N = args.samples
    B = synth.make_batch(N, 32, seed=5)
    cols = np.zeros((N, 40), dtype=np.complex128)
    for k in range(32):  # diode columns idx(k, j, i) of the reference layout; FC columns
        cols[:, k] = B["d"][k]
    for g in range(8):
        cols[:, 32 + g] = B["fc"][g]
    centres = gpd.read_stefan_file(os.path.join(ROOT, "tests", "golden", "Stefan_file.txt"))
    volt = np.empty((N, 80), dtype=np.float32)
    volt[:, 0::2] = (cols + centres[None, :]).real
    volt[:, 1::2] = (cols + centres[None, :]).imag
    for label, t in (("relative", B["t"]), ("mjd", B["t"] + 86400.0 * 60000.5)):
        for window in (None, 1.0):
            ts = []
            for _ in range(args.reps + 1):
                t0 = time.perf_counter()
                out, params, tables = gpd.process_volt(t, volt, offsets=centres, window=window)
                ts.append(time.perf_counter() - t0)
            print(json.dumps({"samples": N, "timestamps": label, "window_s": window,
                              "call_ms": round(1e3 * float(np.median(ts[1:])), 3),
                              "kernels_ms": {k: round(v, 3) for k, v in gpd.timings(0).items()}}),
                  flush=True)


if __name__ == "__main__":
    main()
