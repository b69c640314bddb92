#!/usr/bin/env bash
# r5: deferred π-flip re-fits from 2048 series (fit_defer): records, fit times vs in place.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_parity.py tests/test_gpu_windows.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 7 > $O/probe_defer.jsonl 2> $O/probe_defer.err || { tail -20 $O/probe_defer.err; exit 1; }
GPD_OPTS=fit_defer=0 timeout -k 10 300 python -u tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 7 > $O/probe_inplace.jsonl 2> $O/probe_inplace.err || { tail -20 $O/probe_inplace.err; exit 1; }
cat $O/probe_defer.jsonl $O/probe_inplace.jsonl
