#!/usr/bin/env python3
"""C2 exposure through the host-buffer drop-in (gpd_demodulateall): where the time of one call
goes.  Median of `reps` calls each: the fit alone (records only, gpd_fit_batch), demodulateall
into a fresh output (the reference's semantics: a new matrix per call; once with the previous
result released inside the timed loop, once with every result kept alive and the release timed
apart), the same call into an
output reused across calls (pages already touched), and — for scale — numpy's own
`data.copy()` of the exposure (what `output = copy(data)` costs on one thread).  Then one call
with option host_prof = 1 (the library's wall-clock split on stderr).  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, _p)
import numpy as np  # noqa: E402
import torch  # noqa: E402  (HIP runtime order, as in the tests; pinned host memory)

import gpdemod_loader  # noqa: E402
import synth  # noqa: E402


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(1e3 * float(np.median(ts)), 3)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    gpd = gpdemod_loader.load()
    L = gpd.load()
    gpd.options_from_env()  # GPD_OPTS="name=value,..." (A/B runs, e.g. h2d_parts=1)
    N = 100_000
    B = synth.make_batch(N, 32, seed=42)
    data = np.empty((N, 40), dtype=np.complex128, order="F")
    data[:, :32] = B["d"].T
    fop = np.array([gpd.fc_column_of(c) - 1 for c in range(1, 33)], dtype=np.int32)
    for g in range(8):
        data[:, 32 + g] = B["fc"][g]
    cols = data.T
    t = B["t"]
    out = {}
    out["fit_only_ms"] = med(lambda: gpd.fit_batch(t, cols[:32], cols, fop), reps)
    out["demodulateall_fresh_ms"] = med(lambda: gpd.demodulateall(t, data), reps)
    # the same calls with every result kept until the end: the previous result's release
    # (numpy's munmap of 64 MB of touched pages) then falls outside the timed call
    kept = []
    out["demodulateall_fresh_kept_ms"] = med(lambda: kept.append(gpd.demodulateall(t, data)), reps)
    t0 = time.perf_counter()
    n_kept = len(kept)
    kept.clear()
    out["release_of_one_output_ms"] = round(1e3 * (time.perf_counter() - t0) / n_kept, 3)
    # the exposure in page-locked memory (a caller that pins its buffers): two parts by default
    pin = torch.empty((40, N), dtype=torch.complex128, pin_memory=True).numpy()
    pin[:] = cols
    pdata = pin.T
    out["demodulateall_pinned_kept_ms"] = med(lambda: kept.append(gpd.demodulateall(t, pdata)), reps)
    kept.clear()
    reuse = np.empty((40, N), dtype=np.complex128)
    par = np.zeros(32, dtype=gpd.PARAM_DTYPE)
    import ctypes
    err = ctypes.create_string_buffer(512)

    def call_reuse():
        gpd._lib.check(L.gpd_demodulateall(N, gpd._lib.ptr(t), gpd._lib.ptr(np.ascontiguousarray(cols)), N, None,
                                           None, gpd.GPD_RECENTER, 60, gpd._lib.ptr(par),
                                           gpd._lib.ptr(reuse), N, 1, err, len(err)), err)
    out["demodulateall_reused_output_ms"] = med(call_reuse, reps)
    out["numpy_copy_of_exposure_ms"] = med(lambda: data.copy(order="F"), reps)
    out["numpy_empty_and_touch_ms"] = med(lambda: np.ones((40, N), dtype=np.complex128), reps)
    out["affinity_cpus"] = len(os.sched_getaffinity(0))
    gpd.set_option("host_prof", 1)
    print("--- host_prof: fresh output", file=sys.stderr, flush=True)
    gpd.demodulateall(t, data)
    print("--- host_prof: reused output", file=sys.stderr, flush=True)
    call_reuse()
    print("--- host_prof: pinned input, fresh output", file=sys.stderr, flush=True)
    gpd.demodulateall(t, pdata)
    gpd.set_option("host_prof", 0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
