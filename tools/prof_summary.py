#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>/ (committed evidence).

HBM bytes per k_moments launch = FETCH_SIZE·1024·2 (gfx950 reports ½ of a wide coalesced
stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE·1024, averaged over the headline launches: the
bench command also runs its C2 / C5 blocks, whose moment launches share kernel names, so only the
k_moments launches of the largest grid (the headline workload's) are counted (r5)."""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(path, name):
    with open(path) as f:
        rows = [r for r in csv.DictReader(f)
                if r["Counter_Name"] == name and "k_moments" in r["Kernel_Name"]]
    if not rows:
        return None
    g = max(int(r["Grid_Size"]) for r in rows)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == g]
    return sum(vals) / len(vals)


def headline_moments(trace_csv):
    """Name and mean duration (ms) of the k_moments launches of the largest grid."""
    with open(trace_csv) as f:
        rows = [r for r in csv.DictReader(f) if "k_moments" in r["Kernel_Name"]]
    grid = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    g = max(grid(r) for r in rows)
    top = [r for r in rows if grid(r) == g]
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in top]
    return {"name": top[0]["Kernel_Name"], "calls": len(ms), "avg_ms": sum(ms) / len(ms)}


def main(tag, src=None):
    src = src or os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    bench = json.load(open(os.path.join(src, "bench_trace.json")))
    stats = {}
    with open(os.path.join(dst, "kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
    mom = headline_moments(os.path.join(src, "trace", "run_kernel_trace.csv"))
    fetch_kb = pmc(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write_kb = pmc(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    cfg = bench["config"]
    hbm = fetch_kb * 1024 * 2 + write_kb * 1024
    summary = {
        "tag": tag, "pixels": cfg["series_per_gpu"], "samples": cfg["samples"],
        "k_moments_avg_ms_rocprof": mom["avg_ms"],
        "k_moments_avg_ms_hip_events": bench["roofline"]["avg_ms"],
        "FETCH_SIZE_kB": fetch_kb, "WRITE_SIZE_kB": write_kb,
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes"],
        "traffic_over_algorithmic": hbm / bench["roofline"]["algorithmic_bytes"],
        "bench": bench,
    }
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    storage = cfg.get("storage", "c64")
    name = "pmc_moments.json" if storage == "c64" else f"pmc_moments_{storage}.json"
    if (cfg["series_per_gpu"], cfg["samples"]) != (100_000, 100_000):
        name = name.replace(".json", f"_{cfg['series_per_gpu']}x{cfg['samples']}.json")
    json.dump({k: summary[k] for k in ("tag", "pixels", "samples", "hbm_bytes_per_launch",
                                       "FETCH_SIZE_kB", "WRITE_SIZE_kB")} | {"storage": storage},
              open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "bench"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
