#!/usr/bin/env bash
# r5: the default bench line on the current tree (all blocks), for the round's numbers.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
