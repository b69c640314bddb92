#!/usr/bin/env bash
# r5: faint tiles taken only whole (the rest deferred to k_moments_fix, no masking): the C5
# faint step, the diagnostics variants for reference, then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 120 python tools/faint_time.py --reps 7 > $O/c5_harm.json 2> $O/c5_harm.err || { tail -20 $O/c5_harm.err; exit 1; }
cat $O/c5_harm.json
for m in 9 10; do
  GPD_LIB=fdiag GPD_OPTS=moments=$m timeout -k 10 120 python tools/faint_time.py --reps 3 > $O/faint_m$m.json 2> $O/faint_m$m.err || { tail -20 $O/faint_m$m.err; exit 1; }
  echo "moments=$m $(python -c "import json;d=json.load(open('$O/faint_m$m.json'));print(d['kernels_ms'])")"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
