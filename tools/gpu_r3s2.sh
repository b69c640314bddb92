#!/usr/bin/env bash
# Round-3 re-entry check: GPU suite on the committed tree, then the C5 faint step at the
# default unit count and at U = 24 / 32 (GPD_UNITS, A/B only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_suite_s2.log 2>&1 || { tail -30 gpurun_out/gpu_suite_s2.log; exit 1; }
tail -2 gpurun_out/gpu_suite_s2.log
for u in "" 24 32; do
  GPD_UNITS=$u timeout -k 10 100 python tools/faint_time.py --reps 5 | sed "s/^/units=$u /" || exit 1
done
