#!/usr/bin/env bash
# r4: GPU suite on the committed default (LDS model cache opt-in, per-evaluation view), then the
# exact evaluator with non-temporal series / phasor / model-cache accesses (GPD_LIB=nt) vs default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for r in 1 2; do
for lib in "" nt; do
  GPD_LIB=$lib timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_$lib$r.json 2>$O/c5_$lib$r.err || { tail -20 $O/c5_$lib$r.err; exit 1; }
  echo "C5 exact lib=$lib"; cat $O/c5_$lib$r.json
  GPD_LIB=$lib timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_$lib$r.jsonl 2> $O/c2_$lib$r.err || { tail -20 $O/c2_$lib$r.err; exit 1; }
  echo "C2 lib=$lib"; grep exact $O/c2_$lib$r.jsonl
done
done
