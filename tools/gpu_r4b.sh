#!/usr/bin/env bash
# r4: phase-scheduled harmonic fit (drive_fit_sched) — harmonic parity tests, A/B against the
# run()-driven fit (libgpdemod_nosched.so), C5 fit time, wave-level phase split (diag build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r4b
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_shards.py tests/test_gpu_faint_stats.py \
    > gpurun_out/r4b/tests.log 2>&1 || { tail -40 gpurun_out/r4b/tests.log; exit 1; }
tail -1 gpurun_out/r4b/tests.log
AB_NOTEST=1 bash tools/ab_fit.sh nosched || exit 1
for lib in "" nosched; do
  GPD_LIB=$lib timeout -k 10 100 python tools/faint_time.py --reps 5 >> gpurun_out/r4b/c5.jsonl || exit 1
done
cat gpurun_out/r4b/c5.jsonl
# C5 moment pass: sample units per series (32 = default for faint series) A/B
for u in 16 24 64; do
  GPD_UNITS=$u timeout -k 10 100 python tools/faint_time.py --reps 5 | sed "s/^/{\"units\": $u, \"r\": /; s/\$/}/" >> gpurun_out/r4b/c5_units.jsonl || exit 1
done
cat gpurun_out/r4b/c5_units.jsonl
# exact evaluator: cohort form (G = 8, persistent, MALL-resident rounds) vs the G = 1 batch path
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "cohort_form" > gpurun_out/r4b/cohort_tests.log 2>&1 || { tail -30 gpurun_out/r4b/cohort_tests.log; exit 1; }
tail -1 gpurun_out/r4b/cohort_tests.log
for c in 0 1; do
  GPD_EXACT_COHORT=$c timeout -k 10 200 python tools/faint_time.py --method exact --reps 2 | sed "s/^/{\"cohort\": $c, \"r\": /; s/\$/}/" >> gpurun_out/r4b/exact.jsonl || exit 1
done
cat gpurun_out/r4b/exact.jsonl
