#!/usr/bin/env bash
# r4: exact evaluator prefetch depth A/B (first pass CR_U 4/6/8, residual UR 4/8 at one wave per
# SIMD): C5 exact and C2 exact / fitoffsets, two rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4j}
mkdir -p $O
for r in 1 2; do
for lib in "" u6 u8 ur8; do
  GPD_LIB=$lib timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_$lib$r.json 2>$O/c5_$lib$r.err || { tail -20 $O/c5_$lib$r.err; exit 1; }
  GPD_LIB=$lib timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_$lib$r.jsonl 2> $O/c2_$lib$r.err || { tail -20 $O/c2_$lib$r.err; exit 1; }
  python - <<PY
import json
c5=json.load(open("$O/c5_$lib$r.json")); c2=[json.loads(l) for l in open("$O/c2_$lib$r.jsonl")]
print(json.dumps({"lib":"$lib","c5_exact":c5["kernels_ms"]["fit_exact"],"c2_exact":[c["kernels_ms"].get("fit_exact") for c in c2 if c["method"]=="exact"]}))
PY
done
done
