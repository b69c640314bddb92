"""C2 exposure (32 diodes × 1e5) through gpd_fit_batch: harmonic (default without offsets) and
the exact evaluator (the fitoffsets default, the reference's `--center fit`), the latter with
each series split over G = 1, 2, 4, 8 workgroups (option exact_g; default 8 for 32 series).
Prints one JSON line per case: host wall time per call (PCIe included) and kernel times."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, _p)
import torch  # noqa: F401,E402  (HIP runtime order, as in the tests)
import gpdemod_loader  # noqa: E402
import synth  # noqa: E402

gpd = gpdemod_loader.load()
OPTS = gpd.options_from_env()  # GPD_OPTS="name=value,..." (A/B runs)
# --mjd: real exposures' timestamps, t = TIME·1e-6 + 86400·MJD (src/GPPupilDemodulation.jl:139),
# so ω t ≈ 3.3e10 rad and every χ² evaluation of the exact path reduces its arguments by
# Payne–Hanek
T0 = 86400.0 * 60000.0 if "--mjd" in sys.argv else 0.0
B = synth.make_batch(100000, 32, seed=42, offsets=True, t0=T0)
args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
GS = ("8",) if "--g8" in sys.argv else ("1", "2", "4", "8")  # --g8: the default split only
cases = [(False, "auto", None)] + [(off, "exact", g) for off in (False, True) for g in GS]
for off, method, g in cases:
    if g is None:
        gpd.set_option("exact_g", 0)
    else:
        gpd.set_option("exact_g", int(g))
    gpd.fit_batch(*args, fitoffsets=off, method=method)
    t0 = time.perf_counter()
    for _ in range(3):
        gpd.fit_batch(*args, fitoffsets=off, method=method)
    print(json.dumps({"lib": os.environ.get("GPD_LIB", ""), "opts": OPTS, "t0": T0, "fitoffsets": off, "method": method, "G": g,
                      "ms": round((time.perf_counter() - t0) / 3 * 1e3, 3),
                      "kernels_ms": {k: round(v, 3) for k, v in gpd.timings(0).items()}}))
