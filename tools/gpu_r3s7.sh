#!/usr/bin/env bash
# Faint fixup with the precomputed cos/sin table of deferred samples: faint tests, C5 timing
# (c64, c32), rocprofv3 trace + FETCH/WRITE PMC of the C5 step, C5 sweep, whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "faint or shards or c32 or states or cohort" > gpurun_out/gpu_faint_s7.log 2>&1 || { tail -40 gpurun_out/gpu_faint_s7.log; exit 1; }
tail -1 gpurun_out/gpu_faint_s7.log
timeout -k 10 100 python tools/faint_time.py --reps 5 || exit 1
timeout -k 10 100 python tools/faint_time.py --reps 5 --c32 || exit 1
timeout -k 10 600 bash tools/pmc_c5.sh r3split > gpurun_out/pmc_c5_r3split.log 2>&1 || { tail -20 gpurun_out/pmc_c5_r3split.log; exit 1; }
timeout -k 10 400 python tools/c5_sweep.py --out gpurun_out/c5_sweep_s7.json > gpurun_out/c5_sweep_s7.log 2>&1 || { tail -20 gpurun_out/c5_sweep_s7.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_suite_s7.log 2>&1 || { tail -40 gpurun_out/gpu_suite_s7.log; exit 1; }
tail -1 gpurun_out/gpu_suite_s7.log
