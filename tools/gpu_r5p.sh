#!/usr/bin/env bash
# r5 round-close evidence (first pass): rocprofv3 kernel trace + stats of the bench command and
# FETCH/WRITE PMC passes on the moment kernel (tools/profile.sh), then smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 1000 bash tools/profile.sh r5final || exit 1
cd "$R" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/prof_r5final/smoke.log 2>&1 || { tail -20 gpurun_out/prof_r5final/smoke.log; exit 1; }
tail -3 gpurun_out/prof_r5final/smoke.log
