#!/usr/bin/env bash
# r4: PMC evidence for the C5 exact evaluator (tools/faint_time.py --method exact): kernel trace
# + stats, FETCH_SIZE, WRITE_SIZE and the L2 hit counters, each in its own pass.
set -euo pipefail
TAG=${1:-r4exact}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/pmc_c5.sh" "$TAG" --method exact "$@"
OUT=$R/gpurun_out/pmc_c5_$TAG
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d "$OUT/pmc_l2" -o pmc -- \
    python3 "$R/tools/faint_time.py" --reps 2 --method exact "$@" > "$OUT/l2.json"
find "$OUT/pmc_l2" -name "*.csv" | sort
