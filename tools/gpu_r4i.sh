#!/usr/bin/env bash
# r4: exact evaluator FAST form (unconditional per-sample loads, exact prefetch counts) vs the
# general form (GPD_EXACT_FAST=0): GPU suite, then C5 exact and C2 exact / fitoffsets timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for r in 1 2; do
for fast in 1 0; do
  GPD_EXACT_FAST=$fast timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_fast$fast$r.json 2>$O/c5_fast$fast$r.err || { tail -20 $O/c5_fast$fast$r.err; exit 1; }
  echo "C5 exact fast=$fast"; cat $O/c5_fast$fast$r.json
  GPD_EXACT_FAST=$fast timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_fast$fast$r.jsonl 2> $O/c2_fast$fast$r.err || { tail -20 $O/c2_fast$fast$r.err; exit 1; }
  echo "C2 fast=$fast"; grep exact $O/c2_fast$fast$r.jsonl
done
done
GPD_FIT_PROF=1 timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > /dev/null 2> $O/c2_prof.err || exit 1
grep "exact fit_prof" $O/c2_prof.err
