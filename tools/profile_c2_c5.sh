#!/usr/bin/env bash
# rocprofv3 kernel traces (stats only, no counters) of the secondary workloads: the C5 faint
# harmonic step (tools/faint_time.py) and the C2 exposure through the exact evaluator with MJD
# timestamps at G = 8 (tools/c2_offsets_timing.py --g8 --mjd).  Output under gpurun_out/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_sec
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/c5" -o run -- \
    python3 "$R/tools/faint_time.py" --reps 5 > "$OUT/c5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/c2" -o run -- \
    python3 "$R/tools/c2_offsets_timing.py" --g8 --mjd > "$OUT/c2.log" 2>&1
find "$OUT" -name "*kernel_stats.csv" | sort
