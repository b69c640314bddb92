#!/usr/bin/env bash
# r5: the multi-lane angle search unrolled by 3 (table loads in flight together) — records must
# keep the r5u hashes (32 2929eb194e0b7afa, 4096 eb89fd1d4d7fde6a, 12500 bf0863430cad9d82, 1e5
# 19c354db589194ce); fit times; NEWUOA split.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 5 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
GPD_LIB=fdiag timeout -k 10 180 python tools/fit_probe.py --pixels 32,12500 --reps 2 --prof > $O/fdiag.jsonl 2> $O/fdiag.err || { tail -20 $O/fdiag.err; exit 1; }
grep "fit_prof per" $O/fdiag.err
