#!/usr/bin/env bash
# r4: LDS model cache for the exact evaluator at G = 8 (C2 one exposure, C5 cohort form):
# exact-path GPU tests, then C2 / C5 exact timings with and without it (GPD_EXACT_LMC), and the
# per-workgroup cycle split (GPD_FIT_PROF).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4f}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_faint_stats.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lmc in 0 1; do
  GPD_EXACT_LMC=$lmc timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_lmc$lmc.jsonl 2> $O/c2_lmc$lmc.err || { tail -20 $O/c2_lmc$lmc.err; exit 1; }
  GPD_EXACT_LMC=$lmc GPD_FIT_PROF=1 timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > /dev/null 2> $O/c2_prof_lmc$lmc.err || { tail -20 $O/c2_prof_lmc$lmc.err; exit 1; }
  echo "C2 lmc=$lmc"; cat $O/c2_lmc$lmc.jsonl; grep "exact fit_prof" $O/c2_prof_lmc$lmc.err | tail -2
done
timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_default.json 2>$O/c5_default.err || { tail -20 $O/c5_default.err; exit 1; }
echo "C5 default"; cat $O/c5_default.json
for lmc in 0 1; do
  GPD_EXACT_COHORT=1 GPD_EXACT_LMC=$lmc timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_coh_lmc$lmc.json 2>$O/c5_coh_lmc$lmc.err || { tail -20 $O/c5_coh_lmc$lmc.err; exit 1; }
  echo "C5 cohort lmc=$lmc"; cat $O/c5_coh_lmc$lmc.json
  GPD_EXACT_COHORT=1 GPD_EXACT_LMC=$lmc GPD_FIT_PROF=1 timeout -k 10 150 python tools/faint_time.py --method exact --reps 1 > /dev/null 2>$O/c5_coh_prof_lmc$lmc.err || { tail -20 $O/c5_coh_prof_lmc$lmc.err; exit 1; }
  grep "exact fit_prof" $O/c5_coh_prof_lmc$lmc.err | tail -1
done
