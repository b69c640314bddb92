"""Generate tests/golden/oracle_fits.json — regression fixtures of the CPU oracle.

The reference (Julia) cannot run in this container and ships no fixtures, so these
vectors are produced by the oracle restatement itself from seeded synthetic inputs; they pin the
oracle (and, through tests/test_gpu_parity.py, the GPU path) against silent drift.
Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

CASES = [
    {"name": "C1_one_diode_10k", "N": 10000, "P": 1, "seed": 1},
    {"name": "small_batch", "N": 3000, "P": 8, "seed": 2},
    {"name": "offsets", "N": 3000, "P": 4, "seed": 3, "offsets": True},
    {"name": "recenter_false_xinit", "N": 3000, "P": 4, "seed": 4, "recenter": False,
     "xinit": [0.8, 0.5]},
    {"name": "mjd_t0", "N": 3000, "P": 4, "seed": 5, "t0": 86400.0 * 60000.0},
    {"name": "faint_onlyhigh", "N": 4000, "P": 4, "seed": 6, "faint": True, "onlyhigh": True},
]


def states(N):
    st = np.full(N, 2, dtype=np.int8)
    for k in range(N // 800):
        a = 400 + k * 800
        st[a:a + 200] = 3
        st[a:a + 4] = -1
        st[a + 200:a + 500] = 1
        st[a + 200:a + 212] = -1
    return st


def case_inputs(spec):
    """(batch, states or None, xinit or None) of a fixture case — shared with the GPU test."""
    import synth

    B = synth.make_batch(spec["N"], spec["P"], seed=spec["seed"], t0=spec.get("t0", 0.0),
                         offsets=spec.get("offsets", False))
    st = states(spec["N"]) if spec.get("faint") else None
    if st is not None:
        B["d"] = B["d"] * np.where(st == 3, 1.1, np.where(st == 1, 0.3, 0.6))[None, :]
    xi = np.array(spec["xinit"]) if "xinit" in spec else None
    return B, st, xi


def run_case(oracle, spec):
    B, st, xi = case_inputs(spec)
    flags = oracle.RECENTER if spec.get("recenter", True) else 0
    if spec.get("offsets"):
        flags |= oracle.FIT_OFFSETS
    if spec.get("onlyhigh"):
        flags |= oracle.ONLY_HIGH
    par = oracle.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], state=st, xinit=xi,
                           flags=flags, nthreads=1)
    return {"b": par["b"].tolist(), "phi": par["phi"].tolist(), "chi2": par["chi2"].tolist(),
            "a_re": par["a"].real.tolist(), "a_im": par["a"].imag.tolist(),
            "c_re": par["c"].real.tolist(), "c_im": par["c"].imag.tolist(),
            "nfev": par["nfev"].tolist(), "status": par["status"].tolist()}


if __name__ == "__main__":
    import oracle

    out = {"generator": "tests/golden/make_golden.py (oracle restatement; parity unpinned)",
           "cases": [{"spec": c, "expect": run_case(oracle, c)} for c in CASES]}
    with open(os.path.join(HERE, "oracle_fits.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(CASES), "cases")
