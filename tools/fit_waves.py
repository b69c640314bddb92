"""Summarise the harmonic fit's per-wave timeline (diagnostics build, option fit_prof = 1:
the library prints one `fitwave <w> <start> <end> <max nfev> <hw id>` line per wave, times in
s_memrealtime ticks of 10 ns).  Reads the stderr capture of `tools/fit_probe.py --prof` and prints,
per probe call, the kernel span, the wave-duration distribution, how the span splits into the
waves' rounds on their SIMD slots, and how a wave's duration follows its lanes' largest
evaluation count.

    python tools/fit_waves.py gpurun_out/r5ab/prof.txt [--json out.json]
"""
import argparse
import json
import re
import sys

import numpy as np

TICK_US = 0.01  # s_memrealtime: 100 MHz


def parse(path):
    runs, cur = [], None
    for line in open(path):
        if line.startswith("--- prof"):
            cur = {"title": line.strip()[4:], "waves": []}
            runs.append(cur)
        elif line.startswith("fitwave") and cur is not None:
            _, w, t0, t1, nf, hw = line.split()
            cur["waves"].append((int(w), int(t0), int(t1), int(nf), int(hw, 16)))
    return [r for r in runs if r["waves"]]


def slot_of(hw):
    h = hw & 0xFFFFFFFF
    xcc = (hw >> 32) & 0xF
    simd = (h >> 4) & 3
    cu = (h >> 8) & 0xF
    sh = (h >> 12) & 1
    se = (h >> 13) & 7
    return (xcc, se, sh, cu, simd)


def summarise(run):
    a = np.array([w[1:4] for w in run["waves"]], dtype=np.float64)
    ok = a[:, 1] > 0
    a = a[ok]
    hws = [w[4] for w, k in zip(run["waves"], ok) if k]
    t0 = a[:, 0].min()
    st, en, nf = (a[:, 0] - t0) * TICK_US, (a[:, 1] - t0) * TICK_US, a[:, 2]
    dur = en - st
    slots = {}
    for i, hw in enumerate(hws):
        slots.setdefault(slot_of(hw), []).append(i)
    per_slot = np.array([len(v) for v in slots.values()])
    slot_end = np.array([en[v].max() for v in slots.values()])
    slot_busy = np.array([dur[v].sum() for v in slots.values()])
    q = lambda x, p: float(np.percentile(x, p))
    out = {
        "title": run["title"],
        "waves": int(len(dur)),
        "slots": len(slots),
        "waves_per_slot": {str(k): int((per_slot == k).sum()) for k in sorted(set(per_slot))},
        "span_us": float(en.max()),
        "last_start_us": float(st.max()),
        "duration_us": {"mean": float(dur.mean()), "p10": q(dur, 10), "p50": q(dur, 50),
                        "p90": q(dur, 90), "p99": q(dur, 99), "max": float(dur.max())},
        "slot_busy_us": {"mean": float(slot_busy.mean()), "max": float(slot_busy.max())},
        "slot_end_us": {"p50": q(slot_end, 50), "p90": q(slot_end, 90), "max": float(slot_end.max())},
        "ideal_us": float(dur.sum() / max(1, len(slots))),  # total wave time over the slots
    }
    # duration against the wave's largest evaluation count
    by = {}
    for n, d in zip(nf, dur):
        by.setdefault(int(n), []).append(d)
    out["duration_by_max_nfev"] = {str(k): [len(v), float(np.mean(v))] for k, v in sorted(by.items())}
    # the slots that end last: their waves
    worst = np.argsort(slot_end)[-3:]
    keys = list(slots.keys())
    out["last_slots"] = [[[float(st[i]), float(en[i]), int(nf[i])] for i in slots[keys[j]]] for j in worst]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--json")
    args = ap.parse_args()
    res = [summarise(r) for r in parse(args.path)]
    for r in res:
        print(json.dumps(r))
    if args.json:
        json.dump(res, open(args.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
