#!/usr/bin/env bash
# r4: exact evaluator without the model cache (GPD_EXACT_MCACHE=0: the residual pass evaluates
# the batched model again, 66 instead of 82 B per sample-evaluation) vs with it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4p}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fast_loads or every_split" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for mc in 0 1; do
  GPD_EXACT_MCACHE=$mc timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_mc$mc$r.json 2>$O/c5_mc$mc$r.err || { tail -20 $O/c5_mc$mc$r.err; exit 1; }
  GPD_EXACT_MCACHE=$mc timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_mc$mc$r.jsonl 2> $O/c2_mc$mc$r.err || { tail -20 $O/c2_mc$mc$r.err; exit 1; }
  python - <<PY
import json
c5=json.load(open("$O/c5_mc$mc$r.json")); c2=[json.loads(l) for l in open("$O/c2_mc$mc$r.jsonl")]
print(json.dumps({"mcache":$mc,"c5_exact":c5["kernels_ms"]["fit_exact"],"c2_exact":[c["kernels_ms"].get("fit_exact") for c in c2 if c["method"]=="exact"]}))
PY
done
done
