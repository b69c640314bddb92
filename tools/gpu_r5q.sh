#!/usr/bin/env bash
# r5: what the faint moment kernel's extras cost — the production faint kernel vs its timing
# variants without the fused statistics (moments=9) and without masking (moments=10), and the
# non-faint kernel on the same 4096 × 1e5 shape (diagnostics build; results of 9/10 invalid).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5q
mkdir -p $O
for m in 0 9 10; do
  GPD_LIB=fdiag GPD_OPTS=moments=$m timeout -k 10 120 python tools/faint_time.py --reps 5 > $O/faint_m$m.json 2> $O/faint_m$m.err || { tail -20 $O/faint_m$m.err; exit 1; }
  echo "moments=$m $(python -c "import json;d=json.load(open('$O/faint_m$m.json'));print(d['kernels_ms'])")"
done
timeout -k 10 120 python tools/fit_probe.py --pixels 4096 --reps 5 > $O/plain.jsonl 2> $O/plain.err || exit 1
cat $O/plain.jsonl
