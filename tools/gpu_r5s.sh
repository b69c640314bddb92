#!/usr/bin/env bash
# r5: XCD-aware series order of the exact fit (an FC group's 4 series on one XCD): C5 exact,
# the exact-path GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 300 python tools/faint_time.py --method exact --reps 3 > $O/c5_exact.json 2> $O/c5_exact.err || { tail -20 $O/c5_exact.err; exit 1; }
cat $O/c5_exact.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "exact or faint or oracle or soak" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
