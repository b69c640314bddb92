#!/usr/bin/env bash
# A/B of the fit kernels (GPD_LIB variants, build.py --variant): C4 rank (12 500 series) and C3
# bench steps, plus the harmonic parity tests with the release library.  → gpurun_out/ab_fit/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_fit
mkdir -p "$OUT"
cd "$R"
[ -n "$AB_NOTEST" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_windows.py tests/test_gpu_c4.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for rep in 1 2; do
  for lib in "" "$@"; do
    GPD_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 --pixels 12500 \
        | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','shape':'c4rank','ms':round(j['ms_per_step'],3),'k':j['kernels_ms']}))" >> "$OUT/ab.jsonl" || exit 1
    GPD_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 \
        | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','shape':'c3','ms':round(j['ms_per_step'],3),'k':j['kernels_ms']}))" >> "$OUT/ab.jsonl" || exit 1
  done
done
cat "$OUT/ab.jsonl"
# wave-level phase split of the fit (diagnostics build) on the C4 rank
GPD_LIB=diag GPD_FIT_PROF=1 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --no-f64 --pixels 12500 > "$OUT/fitprof_c4.json" 2> "$OUT/fitprof_c4.err" || exit 1
grep fit_prof "$OUT/fitprof_c4.err" | tail -3
# exact evaluator on the C5 batch (AB_EXACT=1): release vs a 2-waves/SIMD build, + fp32
[ -n "$AB_EXACT" ] || exit 0
for lib in "" minb2; do
  GPD_LIB=$lib timeout -k 10 200 python tools/faint_time.py --method exact --reps 2 >> "$OUT/exact.jsonl" 2>/dev/null || exit 1
done
timeout -k 10 200 python tools/faint_time.py --method fp32 --reps 2 >> "$OUT/exact.jsonl" 2>/dev/null || exit 1
cat "$OUT/exact.jsonl"
