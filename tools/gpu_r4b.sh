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
