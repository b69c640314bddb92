#!/usr/bin/env python3
"""Randomised soak of the other entry points (GPU box), against the oracle or the one-device run,
bit for bit:
  * windows  — gpd_fit_windows with the exact evaluator vs the oracle on every window's slice
               (random N, window length, series, faint states, flags);
  * c32      — ComplexF32 series / FC (gpd_fit_batch_c32) with the exact evaluator vs the oracle
               on the same values widened to ComplexF64;
  * faint    — gpd_mean_var_power (m, w per series and state) vs the oracle's
               compute_mean_var_power restatement, random state runs, onlyhigh;
  * shards   — gpd_fit_batch(n_gpus = 2..5) with option fake_gpus = 1 (shard g on device g mod 1)
               vs n_gpus = 1, automatic method, demodulated output included;
  * mixed    — windows × ComplexF32 × faint × fitoffsets × MJD-scale t0 × device shards, exact
               evaluator, against the oracle per window slice.
Runs until --seconds have passed; one JSON line per case; exits non-zero on the first failure.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--seed", type=int, default=11)
    args = ap.parse_args()
    import numpy as np

    import gpdemod_loader
    import oracle
    import synth
    from test_gpu_parity import assert_exact_bitwise

    gpd = gpdemod_loader.load()
    gpd.set_option("fake_gpus", 1)
    gpd.load()
    oracle.build()
    rng = np.random.default_rng(args.seed)

    def states(N):
        st = np.empty(N, np.int8)
        i = 0
        while i < N:
            n = int(rng.integers(1, max(2, N // 5)))
            st[i:i + n] = rng.choice([3, 2, 1, -1], p=[0.3, 0.3, 0.3, 0.1])
            i += n
        return st

    def flags(recenter, fitoffsets, onlyhigh):
        return ((oracle.RECENTER if recenter else 0) | (oracle.FIT_OFFSETS if fitoffsets else 0)
                | (oracle.ONLY_HIGH if onlyhigh else 0))

    counts = {"windows": 0, "c32": 0, "faint": 0, "shards": 0, "mixed": 0}
    t_end = time.time() + args.seconds
    case = 0
    while time.time() < t_end:
        case += 1
        kind = ["windows", "c32", "faint", "shards", "mixed"][case % 5]
        t1 = time.time()
        desc = {"case": case, "kind": kind}
        try:
            if kind == "windows":
                N = int(rng.integers(2, 9000))
                w = int(rng.choice([2, 3, 100, 255, 256, 500, 1500, int(rng.integers(2, N + 1))]))
                C = int(rng.integers(1, 17))
                B = synth.make_batch(N, C, seed=int(rng.integers(1, 1 << 30)),
                                     offsets=bool(rng.random() < 0.3))
                rec, off, oh = bool(rng.random() < 0.8), bool(rng.random() < 0.3), False
                st = None
                if rng.random() < 0.35:
                    st, oh = states(N), bool(rng.random() < 0.4)
                desc.update(N=N, window=w, C=C, faint=st is not None, fitoffsets=off)
                got = gpd.fit_windows(B["t"], B["d"], B["fc"], B["fc_of_pixel"], w, state=st,
                                      recenter=rec, fitoffsets=off, onlyhigh=oh, method="exact")
                ref = []
                for s0 in range(0, N, w):
                    I = slice(s0, min(N, s0 + w))
                    ref.append(oracle.fit_batch(B["t"][I], B["d"][:, I], B["fc"][:, I],
                                                B["fc_of_pixel"],
                                                state=None if st is None else st[I],
                                                flags=flags(rec, off, oh)))
                ref = np.stack(ref)
                assert got.shape == ref.shape, (got.shape, ref.shape)
                assert_exact_bitwise(got.reshape(-1), ref.reshape(-1), label=json.dumps(desc))
            elif kind == "c32":
                N = int(rng.integers(2, 20000))
                P = int(rng.integers(1, 33))
                B = synth.make_batch(N, P, seed=int(rng.integers(1, 1 << 30)),
                                     group=int(rng.choice([1, 2, 4])),
                                     offsets=bool(rng.random() < 0.3))
                d32, f32 = B["d"].astype(np.complex64), B["fc"].astype(np.complex64)
                rec, off = bool(rng.random() < 0.8), bool(rng.random() < 0.3)
                st, oh = (states(N), bool(rng.random() < 0.4)) if rng.random() < 0.3 else (None, False)
                desc.update(N=N, P=P, faint=st is not None, fitoffsets=off)
                got = gpd.fit_batch(B["t"], d32, f32, B["fc_of_pixel"], state=st, recenter=rec,
                                    fitoffsets=off, onlyhigh=oh, method="exact")
                ref = oracle.fit_batch(B["t"], d32.astype(np.complex128), f32.astype(np.complex128),
                                       B["fc_of_pixel"], state=st, flags=flags(rec, off, oh))
                assert_exact_bitwise(got, ref, label=json.dumps(desc))
            elif kind == "faint":
                N = int(rng.integers(2, 50000))
                P = int(rng.integers(1, 9))
                d = (rng.normal(size=(P, N)) + 1j * rng.normal(size=(P, N))) * rng.uniform(0.01, 10)
                st = states(N)
                oh = bool(rng.random() < 0.4)
                desc.update(N=N, P=P, onlyhigh=oh)
                m5, w5 = gpd.mean_var_power_batch(st, d, onlyhigh=oh)
                for k in range(P):
                    rm, rw = oracle.mean_var_power_series(st, d[k], onlyhigh=oh)
                    same = ((m5[k] == rm) | (np.isnan(m5[k]) & np.isnan(rm))) & \
                        ((w5[k] == rw) | (np.isnan(w5[k]) & np.isnan(rw)))
                    assert same.all(), f"{desc}: series {k}: m {m5[k]} vs {rm}, w {w5[k]} vs {rw}"
            elif kind == "mixed":
                # windows × ComplexF32 × faint × fitoffsets × MJD-scale t0 × device shards,
                # exact evaluator, against the oracle per window slice on the widened values
                N = int(rng.integers(2, 6000))
                w = int(rng.choice([2, 100, 300, int(rng.integers(2, N + 1))]))
                C = int(rng.integers(1, 13))
                t0 = float(rng.choice([0.0, 86400.0 * 60000.5]))
                B = synth.make_batch(N, C, seed=int(rng.integers(1, 1 << 30)), t0=t0,
                                     offsets=bool(rng.random() < 0.4))
                c32 = bool(rng.random() < 0.5)
                d, fc = B["d"], B["fc"]
                if c32:
                    d, fc = d.astype(np.complex64), fc.astype(np.complex64)
                rec, off = bool(rng.random() < 0.8), bool(rng.random() < 0.4)
                st, oh = (states(N), bool(rng.random() < 0.4)) if rng.random() < 0.4 else (None, False)
                ng = int(rng.integers(1, 4))
                desc.update(N=N, window=w, C=C, t0=t0, c32=c32, faint=st is not None,
                            fitoffsets=off, n_gpus=ng)
                got = gpd.fit_windows(B["t"], d, fc, B["fc_of_pixel"], w, state=st, recenter=rec,
                                      fitoffsets=off, onlyhigh=oh, method="exact", n_gpus=ng)
                d64, f64 = d.astype(np.complex128), fc.astype(np.complex128)
                ref = np.stack([oracle.fit_batch(B["t"][I], d64[:, I], f64[:, I], B["fc_of_pixel"],
                                                 state=None if st is None else st[I],
                                                 flags=flags(rec, off, oh))
                                for I in (slice(s0, min(N, s0 + w)) for s0 in range(0, N, w))])
                assert_exact_bitwise(got.reshape(-1), ref.reshape(-1), label=json.dumps(desc))
            else:
                N = int(rng.integers(2, 20000))
                P = int(rng.integers(1, 60))
                ng = int(rng.integers(2, 6))
                B = synth.make_batch(N, P, seed=int(rng.integers(1, 1 << 30)),
                                     group=int(rng.choice([1, 2, 4])))
                st = states(N) if rng.random() < 0.3 else None
                method = str(rng.choice(["auto", "exact", "harmonic"])) if N >= 256 else "exact"
                desc.update(N=N, P=P, n_gpus=ng, method=method, faint=st is not None)
                one, o1 = gpd.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], state=st,
                                        method=method, want_output=True)
                many, om = gpd.fit_batch(B["t"], B["d"], B["fc"], B["fc_of_pixel"], state=st,
                                         method=method, want_output=True, n_gpus=ng)
                assert one.tobytes() == many.tobytes(), f"{desc}: records differ across shards"
                assert o1.tobytes() == om.tobytes(), f"{desc}: demodulated output differs"
        except AssertionError as e:
            print("FAIL", json.dumps(desc), e, flush=True)
            return 1
        counts[kind] += 1
        print(json.dumps({**desc, "ok": True, "s": round(time.time() - t1, 2)}), flush=True)
    print(f"soak_more: {case} cases, all bit-identical: {json.dumps(counts)}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
