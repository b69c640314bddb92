"""C2 exposure (32 diodes x 1e5) through gpd_fit_batch with and without fitoffsets (the
exact evaluator is the fitoffsets default): wall time per call and kernel times."""
import sys, time, json
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, 'tests')):
    sys.path.insert(0, _p)
import torch  # noqa
import numpy as np
import gpdemod_loader, synth
gpd = gpdemod_loader.load()
B = synth.make_batch(100000, 32, seed=42, offsets=True)
args = (B["t"], B["d"], B["fc"], B["fc_of_pixel"])
for off in (False, True):
    gpd.fit_batch(*args, fitoffsets=off)
    t0 = time.perf_counter()
    for _ in range(3):
        gpd.fit_batch(*args, fitoffsets=off)
    print(json.dumps({"fitoffsets": off, "ms": (time.perf_counter() - t0) / 3 * 1e3,
                      "kernels": gpd.timings(0)}))
