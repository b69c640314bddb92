#!/usr/bin/env bash
# r5 first GPU pass: the GPU suite (in-place demodulated output, per-rank bench diagnostics,
# faint fallback statistics test), smoke(), and the default bench line (C2 exposure block).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['kernels_ms'], j['c4_rank_rehearsal']['kernels_ms'], j['c5_faint']['gpu']['ms_per_step'], json.dumps(j['c2_exposure']['cases']))"
