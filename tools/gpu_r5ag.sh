#!/usr/bin/env bash
# r5 round close (after the deferred re-fits): the default bench line, rocprofv3 kernel trace/stats + FETCH/WRITE PMC of the
# bench command (tools/profile.sh), smoke — all on the final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5ag
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 1000 bash tools/profile.sh r5ag || exit 1
cd "$R" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
