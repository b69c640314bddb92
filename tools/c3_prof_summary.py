#!/usr/bin/env python3
"""C3 moment-kernel evidence from a tools/profile.sh run (the bench command also runs the C2 and
C5 blocks, whose k_moments launches share kernel names with C3's): picks the C3 launches of
k_moments_ws<0,false,c64,2,true,false> by their grid (1e5 series → 782 × 13 workgroups of 512
threads), and writes profiles/<tag>/summary.json with the launches' trace durations, the bench's
own HIP-event average, the FETCH_SIZE / WRITE_SIZE PMC per launch and the corrected HBM traffic
(FETCH_SIZE·1024·2 + WRITE_SIZE·1024, MI355X_MICROARCH.md §HBM), plus the fit kernels' medians.

    python tools/c3_prof_summary.py <tag> <prof dir> [command text]
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C3_KERNEL = "k_moments_ws<0, false, gpd::c64, 2, true, false>"


def c3_grid(grid):
    return grid >= 782 * 13 * 512  # the C3 launch's threads (C2 / C5 / C4-rank launches are far fewer)


def main(tag, src, command=""):
    dst = os.path.join(ROOT, "profiles", tag)
    trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    c3 = [r for r in trace if C3_KERNEL in r["Kernel_Name"]
          and c3_grid(int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]))]
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in c3]
    bench = json.loads(open(os.path.join(src, "bench_trace.json")).read().strip().splitlines()[-1])

    def pmc(sub, name):
        rows = csv.DictReader(open(os.path.join(src, sub, "pmc_counter_collection.csv")))
        return [float(r["Counter_Value"]) for r in rows
                if r["Counter_Name"] == name and C3_KERNEL in r["Kernel_Name"]
                and c3_grid(int(r["Grid_Size"]))]

    fetch, write = pmc("pmc_fetch", "FETCH_SIZE"), pmc("pmc_write", "WRITE_SIZE")
    traffic = statistics.mean(fetch) * 1024 * 2 + statistics.mean(write) * 1024
    alg = bench["roofline"]["algorithmic_bytes"]
    fits = {}
    for r in trace:
        if "k_fit_harmonic" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0]
            fits.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {
        "command": command or f"tools/profile.sh {tag}",
        "build_id": bench.get("build_id"),
        "c3_moment_kernel": "k_moments_ws<0,false,c64,2,true,false> on 1e5 x 1e5",
        "c3_launch_ms_trace": [round(x, 3) for x in ms],
        "c3_timed_launch_mean_ms": round(statistics.mean(ms[1:] if len(ms) > 1 else ms), 3),
        "bench_in_run_hip_events_avg_ms_same_run": bench["roofline"]["avg_ms"],
        "pmc_fetch_size_kb_per_launch": fetch,
        "pmc_write_size_kb_per_launch": write,
        "traffic_bytes_per_launch_corrected": round(traffic),
        "algorithmic_bytes": alg,
        "traffic_over_algorithmic": round(traffic / alg, 4),
        "fit_harmonic_median_ms": {k: round(statistics.median(v), 4) for k, v in fits.items()},
    }
    json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
