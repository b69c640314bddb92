#!/usr/bin/env bash
# r5: faint producers without masking on whole one-state tiles + select-free fs_abs: faint
# parity tests, the C5 faint step; then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "faint or demodulateall or shard" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/faint_time.py --reps 7 > $O/c5_harm.json 2> $O/c5_harm.err || { tail -20 $O/c5_harm.err; exit 1; }
cat $O/c5_harm.json
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 2500 $O/bench.json
