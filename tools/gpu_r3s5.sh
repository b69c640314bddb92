#!/usr/bin/env bash
# State-split faint moments, fixup launched before the moment pass: faint tests, C5 timing,
# rocprofv3 trace + FETCH/WRITE PMC passes of the C5 step (tools/pmc_c5.sh r3split).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "faint or shards or c32 or states or cohort" > gpurun_out/gpu_faint_s5.log 2>&1 || { tail -40 gpurun_out/gpu_faint_s5.log; exit 1; }
tail -1 gpurun_out/gpu_faint_s5.log
timeout -k 10 100 python tools/faint_time.py --reps 5 || exit 1
timeout -k 10 100 python tools/faint_time.py --reps 5 --c32 || exit 1
timeout -k 10 600 bash tools/pmc_c5.sh r3split > gpurun_out/pmc_c5_r3split.log 2>&1 || { tail -20 gpurun_out/pmc_c5_r3split.log; exit 1; }
timeout -k 10 600 bash tools/pmc_c5.sh r3split_c32 --c32 > gpurun_out/pmc_c5_r3split_c32.log 2>&1 || { tail -20 gpurun_out/pmc_c5_r3split_c32.log; exit 1; }
echo done
