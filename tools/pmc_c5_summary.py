#!/usr/bin/env python3
"""Summarise tools/pmc_c5.sh runs (gpurun_out/pmc_c5_<tag>/) into one JSON: per kernel of the C5
faint harmonic step, the rocprofv3 average duration and the HBM bytes per launch from the
separate FETCH_SIZE / WRITE_SIZE passes — FETCH_SIZE doubled (gfx950 reports ½ of a wide
coalesced read, MI355X_MICROARCH.md §HBM), WRITE_SIZE as is — per complex sample of the batch.
Usage: tools/pmc_c5_summary.py <out.json> <tag> [<tag> ...]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = ("k_faint_p1", "k_faint_p2", "k_faint_fin", "k_moments_ws", "k_reduce_moments", "k_fit_exact",
        "k_fit_harmonic", "k_prepare", "k_table", "k_faint_defer", "k_fix_table", "k_moments_fix",
        "k_faint_fused_fin")


def short(name):
    return next((k for k in KEEP if k in name), None)


def main(out, tags):
    res = {"what": __doc__.split("\n\n")[0], "runs": {}}
    for tag in tags:
        src = os.path.join(ROOT, "gpurun_out", f"pmc_c5_{tag}")
        meta = json.load(open(os.path.join(src, "trace.json")))
        samples = meta["series"] * meta["samples"]
        stats = {}
        for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
            k = short(r["Name"])
            if k:
                stats[k] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
        for cn, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(os.path.join(src, sub, "pmc_counter_collection.csv"))):
                k = short(r["Kernel_Name"])
                if k and r["Counter_Name"] == cn:
                    agg[k].append(float(r["Counter_Value"]))
            for k, v in agg.items():
                kb = sum(v) / len(v)
                b = kb * 1024 * (2 if cn == "FETCH_SIZE" else 1)
                stats.setdefault(k, {})[cn.lower() + "_bytes"] = b
                stats[k][cn.lower() + "_B_per_sample"] = round(b / samples, 3)
        tot = sum(v.get("fetch_size_bytes", 0) + v.get("write_size_bytes", 0) for v in stats.values())
        ms = sum(v.get("avg_ms", 0) for v in stats.values())
        esz = 8 if meta.get("c32") else 16
        algo = samples * (esz + esz / 4) + 9 * meta["samples"]
        res["runs"][tag] = {"series": meta["series"], "samples": meta["samples"],
                            "storage": "c32" if meta.get("c32") else "c64", "kernels": stats,
                            "step_kernel_ms": round(ms, 3), "hbm_bytes": tot,
                            "hbm_B_per_sample": round(tot / samples, 2),
                            "algorithmic_B_per_sample": round(algo / samples, 2),
                            "traffic_over_algorithmic": round(tot / algo, 3),
                            "achieved_frac_of_8TBs_algorithmic": round(algo / (ms * 1e-3) / 8e12, 4)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({t: {k: v for k, v in r.items() if k != "kernels"} for t, r in res["runs"].items()},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
