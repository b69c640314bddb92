#!/usr/bin/env bash
# One GPU job of round evidence (run through gpurun): the GPU suite, smoke(), the default bench
# line and the rocprofv3 evidence of the bench command (tools/profile.sh: kernel trace + stats,
# then separate FETCH_SIZE / WRITE_SIZE PMC passes), every step under its own time limit, chained
# so that a failing step ends the job.  Replaces the one-off gpu_r*.sh scripts of rounds 3-5.
# Usage: tools/gpu_round.sh <tag> [steps...]   steps: suite smoke bench prof (default: all)
set -euo pipefail
TAG=${1:?tag}; shift
STEPS=${*:-suite smoke bench prof}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for s in $STEPS; do
  case $s in
    suite)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > "$OUT/gpu_suite.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    prof)
      timeout -k 10 900 bash tools/profile.sh "$TAG" > "$OUT/prof_files.txt" 2>&1 ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
  echo "step $s done" >> "$OUT/steps.log"
done
