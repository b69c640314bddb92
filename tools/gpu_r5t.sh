#!/usr/bin/env bash
# r5: the fit's moment source (LDS copy vs L2) and shape invariance tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
