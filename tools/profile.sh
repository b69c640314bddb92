#!/usr/bin/env bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun):
#   1) kernel trace + stats of the bench command (per-kernel average durations)
#   2) separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the moment kernel — never combined with
#      tracing domains (MI355X_MICROARCH.md §rocprofv3; gpurun policy).
# Usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-r1}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS=("$@")
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-f64 --no-c4 --sustain 0 "${ARGS[@]}" > "$OUT/bench_trace.json"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_moments -f csv -d "$OUT/pmc_fetch" -o pmc -- \
    python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu --no-f64 --no-c4 --sustain 0 "${ARGS[@]}" > "$OUT/bench_pmc_fetch.json"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_moments -f csv -d "$OUT/pmc_write" -o pmc -- \
    python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu --no-f64 --no-c4 --sustain 0 "${ARGS[@]}" > "$OUT/bench_pmc_write.json"
find "$OUT" -name "*.csv" | sort
