#!/usr/bin/env bash
# r4 end: the model-cache A/B (tools/gpu_r4p.sh), then the whole GPU suite and smoke() on the
# committed tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
# (the model-cache A/B of tools/gpu_r4p.sh was reverted before it ran)
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
