#!/usr/bin/env bash
# r5: NEWUOA's subroutines out of line (trsapp, biglag, bigden, update, shift_base) — records
# must keep the r5u hashes (32 2929eb194e0b7afa, 4096 eb89fd1d4d7fde6a, 12500 bf0863430cad9d82,
# 1e5 19c354db589194ce); fit and exact-path times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 5 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
timeout -k 10 300 python tools/faint_time.py --method exact --reps 2 > $O/c5_exact.json 2> $O/c5_exact.err || { tail -20 $O/c5_exact.err; exit 1; }
cat $O/c5_exact.json
timeout -k 10 120 python tools/c2_offsets_timing.py > $O/c2_exact.jsonl 2> $O/c2_exact.err || { tail -20 $O/c2_exact.err; exit 1; }
cat $O/c2_exact.jsonl
