#!/usr/bin/env bash
# A/B of the harmonic fit's occupancy (r6): the release library against a build whose
# k_fit_harmonic allows two waves per SIMD (build.py --variant minw2 -DGPD_FIT_MINW=2), each at
# the automatic series-per-wave and at about half of it (so the waves double and pair up on the
# SIMDs); plus the C5 step with the release library (records hash, per-kernel times).
# Usage: tools/ab_fit_occ.sh [variant]   → gpurun_out/ab_fit_occ/
set -o pipefail
V=${1:-minw2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_fit_occ
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_faint_stats.py tests/test_gpu_parity.py -k "faint or defer or fix" > "$OUT/tests.log" 2>&1 \
    || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 120 python tools/faint_time.py --reps 5 | sed "s/^/lib= /" >> "$OUT/c5.txt" || exit 1
for rep in 1 2; do
  for lib in "" "$V"; do
    GPD_LIB=$lib timeout -k 10 200 python tools/fit_probe.py --pixels 32,4096,12500 --lanes 0,2,7 --reps 5 \
        | sed "s/^/lib=$lib rep=$rep /" >> "$OUT/fit.txt" || exit 1
    GPD_LIB=$lib GPD_OPTS=fit_lanes=2 timeout -k 10 120 python tools/faint_time.py --reps 5 \
        | sed "s/^/lib=$lib lanes=2 /" >> "$OUT/c5.txt" || exit 1
  done
done
cat "$OUT/c5.txt" "$OUT/fit.txt"
