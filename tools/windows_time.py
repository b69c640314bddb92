#!/usr/bin/env python3
"""Windowed batch timing (GPU box): one C2 exposure (32 diodes × 1e5 samples at 2 ms, synth seed 5)
in windows of --window samples through gpd_fit_windows (host buffers), per-kernel HIP-event times
of the last of --reps calls and the median wall time of the call.  One JSON line."""
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
    ap.add_argument("--window", type=int, default=500)
    ap.add_argument("--samples", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--method", default="auto")
    args = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (before libgpdemod, as in tests/conftest.py)

    import gpdemod_loader
    import synth

    gpd = gpdemod_loader.load()
    B = synth.make_batch(args.samples, 32, seed=5)
    ts, rec = [], None
    for _ in range(args.reps + 1):
        t0 = time.perf_counter()
        rec = gpd.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], args.window,
                              method=args.method)
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"window": args.window, "series": int(rec.size), "method": args.method,
                      "fit_lanes": gpd.get_option("fit_lanes") or "auto",
                      "call_ms": round(1e3 * float(np.median(ts[1:])), 3),
                      "kernels_ms": {k: round(v, 3) for k, v in gpd.timings(0).items()},
                      "records_sha": __import__("hashlib").sha256(rec.tobytes()).hexdigest()[:16]}))


if __name__ == "__main__":
    main()
