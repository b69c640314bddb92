#!/usr/bin/env bash
# State-split faint moments: faint GPU tests, the C5 step with the statistics beside the moment
# pass (default) and serial (GPD_FAINT_SIDE=0), then the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "faint or shards or c32 or states or cohort" > gpurun_out/gpu_faint_s3.log 2>&1 || { tail -40 gpurun_out/gpu_faint_s3.log; exit 1; }
tail -2 gpurun_out/gpu_faint_s3.log
for side in 1 0; do
  GPD_FAINT_SIDE=$side timeout -k 10 100 python tools/faint_time.py --reps 5 | sed "s/^/side=$side /" || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_suite_s3.log 2>&1 || { tail -40 gpurun_out/gpu_suite_s3.log; exit 1; }
tail -2 gpurun_out/gpu_suite_s3.log
