#!/usr/bin/env bash
# A/B of the exact evaluator (GPD_LIB variants): C2 exposure at G = 8 (with and without
# fitoffsets, tools/c2_offsets_timing.py) and the C5 batch (faint, 4096 × 1e5) exact and fp32.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_exact
mkdir -p "$OUT"
cd "$R"
for lib in "" "$@"; do
  GPD_LIB=$lib timeout -k 10 120 python tools/c2_offsets_timing.py --g8 >> "$OUT/c2.jsonl" 2>/dev/null || exit 1
  for m in exact fp32; do
    GPD_LIB=$lib timeout -k 10 200 python tools/faint_time.py --method $m --reps 2 \
      | python -c "import json,sys; j=json.loads(sys.stdin.read()); j['lib']='$lib'; print(json.dumps(j))" >> "$OUT/c5.jsonl" || exit 1
  done
done
cat "$OUT/c2.jsonl" "$OUT/c5.jsonl"
