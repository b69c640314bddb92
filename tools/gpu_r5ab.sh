#!/usr/bin/env bash
# r5: per-wave timeline of the harmonic fit (diagnostics build) on C3 and a C4 rank.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5ab
mkdir -p $O
GPD_LIB=fdiag timeout -k 10 400 python -u tools/fit_probe.py --pixels 100000,12500 --reps 3 --prof > $O/probe.jsonl 2> $O/prof.txt || { tail -30 $O/prof.txt; exit 1; }
grep -v fitwave $O/prof.txt | tail -20
