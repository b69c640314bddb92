#!/usr/bin/env bash
# r5 round close (deferred re-fits measured and removed): GPU suite, default bench
# line, rocprofv3 kernel trace/stats + FETCH/WRITE PMC (tools/profile.sh), smoke — final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5aj
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
timeout -k 10 700 bash tools/profile.sh r5aj || exit 1
cd "$R" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
