#!/usr/bin/env bash
# New alignment test, smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_shards.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "alignment or faint" > gpurun_out/gpu_align_s8.log 2>&1 || { tail -40 gpurun_out/gpu_align_s8.log; exit 1; }
tail -1 gpurun_out/gpu_align_s8.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
