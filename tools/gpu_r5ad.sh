#!/usr/bin/env bash
# r5: harmonic fit on C3 (1e5 series) against waves per CU (option fit_wpc, LDS reserved) and
# series per wave (fit_lanes): rounds of waves vs the per-wave crowding of the CU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5ad
mkdir -p $O
: > $O/sweep.jsonl
for cfg in "0 0,49" "3 64,44" "2 64,49" "1 56,64"; do
  set -- $cfg
  GPD_OPTS=fit_wpc=$1 timeout -k 10 200 python -u tools/fit_probe.py --pixels 100000 --lanes $2 --reps 5 >> $O/sweep.jsonl 2> $O/err_$1.txt || { tail -20 $O/err_$1.txt; exit 1; }
done
cat $O/sweep.jsonl
