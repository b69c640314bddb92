#!/usr/bin/env bash
# rocprofv3 evidence for the C5 faint harmonic step (tools/faint_time.py: 4096 × 1e5, seed 11):
#   1) kernel trace + stats (per-kernel average durations)
#   2) separate PMC passes FETCH_SIZE and WRITE_SIZE over every kernel of the step (never
#      combined with tracing domains; MI355X_MICROARCH.md §HBM/rocprofv3).
# Usage: tools/pmc_c5.sh <tag> [faint_time.py args...]   → gpurun_out/pmc_c5_<tag>/
set -euo pipefail
TAG=${1:-r3}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_c5_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 "$R/tools/faint_time.py" --reps 5 "$@" > "$OUT/trace.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o pmc -- \
    python3 "$R/tools/faint_time.py" --reps 2 "$@" > "$OUT/fetch.json"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o pmc -- \
    python3 "$R/tools/faint_time.py" --reps 2 "$@" > "$OUT/write.json"
find "$OUT" -name "*.csv" | sort
