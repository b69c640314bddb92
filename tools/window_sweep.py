#!/usr/bin/env python3
"""Harmonic-window parity against the oracle as a function of the window length (GPU box).

processmetrology's windowed mode fits every window of `nwindow` samples on its own
(src/GPPupilDemodulation.jl:191-205; 1-s windows at 500 Hz = 500 samples).  For each window length
w, `--exposures` exposures of 8 windows × 32 diodes are fitted through gpd_fit_windows with the
harmonic evaluator forced (METHOD_HARMONIC is refused below HARM_MIN_SPAN, so the sweep asks
the library's windows API with option harm_min_span = 1, a test override) and by the oracle on every
window's slice, with 12 perturbed oracle runs (χ² × (1 ± 128 ulp)).  Reports per w: the fraction
within 1e-10, the max deviation, the oracle's own envelope, and how many series land beyond
NEWUOA's rhoend (1e-3).  Output: one JSON object (profiles/r3/window_sweep.json)."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", default="200,256,300,345,400,450,500,600,750,1000")
    ap.add_argument("--exposures", type=int, default=4)
    ap.add_argument("--perturb", type=int, default=12)
    args = ap.parse_args()
    import numpy as np

    import gpdemod_loader
    import oracle
    import synth

    gpd = gpdemod_loader.load()
    gpd.set_option("harm_min_span", 1)
    gpd.load()

    def dev(x, r):
        dphi = np.abs((x["phi"] - r["phi"] + np.pi) % (2 * np.pi) - np.pi)
        return np.max([np.abs(x["b"] - r["b"]) / np.abs(r["b"]),
                       dphi / np.maximum(1.0, np.abs(r["phi"])),
                       np.abs(x["a"] - r["a"]) / np.abs(r["a"]),
                       np.abs(x["chi2"] - r["chi2"]) / np.abs(r["chi2"])], axis=0)

    out = {"what": __doc__.split("\n\n")[0], "rows": []}
    for w in [int(x) for x in args.windows.split(",")]:
        got_all, ref_all, pert_all = [], [], [[] for _ in range(args.perturb)]
        for e in range(args.exposures):
            B = synth.make_batch(8 * w, 32, seed=100 + e)
            got = gpd.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], w,
                                  method="harmonic")
            for s0 in range(0, 8 * w, w):
                I = slice(s0, s0 + w)
                a = (B["t"][I], B["d"][:, I], B["fc"][:, I], B["fc_of_pixel"])
                ref_all.append(oracle.fit_batch(*a, flags=oracle.RECENTER))
                for j in range(args.perturb):
                    pert_all[j].append(oracle.fit_batch(*a, flags=oracle.RECENTER,
                                                        perturb_seed=j + 1, perturb_ulps=128.0))
            got_all.append(got.reshape(-1))
        got = np.concatenate(got_all)
        ref = np.concatenate(ref_all)
        pert = [np.concatenate(p) for p in pert_all]
        harm = (got["status"] & gpd.GPD_ST_EXACT) == 0
        e = dev(got, ref)
        env = np.max([dev(p, ref) for p in pert], axis=0)
        row = {"window": w, "series": int(e.size), "harmonic_fits": int(harm.sum()),
               "within_1e-10": round(float((e <= 1e-10).mean()), 4),
               "max_dev": float(e.max()), "median_dev": float(np.median(e)),
               "beyond_1e-3": int((e > 1e-3).sum()),
               "oracle_envelope_max": float(env.max()),
               "oracle_envelope_beyond_1e-3": int((env > 1e-3).sum()),
               "outside_1.5x_envelope": int((e > 1.5 * env + 1e-10).sum())}
        print(json.dumps(row), file=sys.stderr, flush=True)
        out["rows"].append(row)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
