#!/usr/bin/env bash
# r4: exact evaluator split form (two threads per canonical chain at G = 8) vs 256-thread parts:
# exact-path GPU tests, C2 exact / fitoffsets and the C5 cohort form.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4l}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for sp in 1 0; do
  GPD_EXACT_SPLIT=$sp timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_split$sp$r.jsonl 2> $O/c2_split$sp$r.err || { tail -20 $O/c2_split$sp$r.err; exit 1; }
  echo "C2 split=$sp"; grep exact $O/c2_split$sp$r.jsonl
done
done
GPD_EXACT_SPLIT=1 GPD_FIT_PROF=1 timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > /dev/null 2> $O/c2_prof.err || exit 1
grep "exact fit_prof" $O/c2_prof.err
GPD_EXACT_SPLIT=1 GPD_EXACT_COHORT=1 timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_coh_split.json 2>$O/c5_coh_split.err || { tail -20 $O/c5_coh_split.err; exit 1; }
echo "C5 cohort split"; cat $O/c5_coh_split.json
