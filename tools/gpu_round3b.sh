#!/usr/bin/env bash
# round-3 GPU check: the GPU suite, then the exact-path and cohort-pipeline timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/r3b
mkdir -p "$OUT"
cd "$R"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > "$OUT/gpu_suite.log" 2>&1 || { echo SUITE_FAILED; tail -40 "$OUT/gpu_suite.log"; exit 1; }
tail -2 "$OUT/gpu_suite.log"
for w in 1 2; do
  GPD_EXACT_WAVES=$w timeout -k 10 200 python tools/faint_time.py --method exact --reps 2 | sed "s/^/waves$w /" >> "$OUT/exact.txt" || exit 1
done
timeout -k 10 200 python tools/faint_time.py --method fp32 --reps 2 >> "$OUT/exact.txt" || exit 1
timeout -k 10 100 python tools/c2_offsets_timing.py --g8 >> "$OUT/exact.txt" 2>/dev/null || exit 1
for c in 1 2 3 4; do
  GPD_COHORTS=$c timeout -k 10 100 python tools/faint_time.py --reps 5 | sed "s/^/c5 cohorts$c /" >> "$OUT/cohorts.txt" || exit 1
done
for c in 1 2 4; do
  GPD_COHORTS=$c timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 \
     | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('c3 cohorts$c', round(j['ms_per_step'],3), json.dumps(j['kernels_ms']))" >> "$OUT/cohorts.txt" || exit 1
  GPD_COHORTS=$c timeout -k 10 100 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 --pixels 12500 \
     | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('c4rank cohorts$c', round(j['ms_per_step'],3), json.dumps(j['kernels_ms']))" >> "$OUT/cohorts.txt" || exit 1
done
cat "$OUT/exact.txt" "$OUT/cohorts.txt"
