#!/usr/bin/env bash
# r4 close: GPU suite, smoke(), the default bench line, rocprofv3 kernel trace + FETCH/WRITE PMC
# of the C3 moment kernel, and the C5 exact PMC summary inputs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['kernels_ms'], j['sustained']['ms_per_step_mean'], j['c5_faint']['gpu']['ms_per_step'], j['c5_faint']['gpu_exact']['ms_per_step'], j['build_id'])"
bash tools/profile.sh ${TAG:-r4final} --no-c5 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -2 $O/profile.log
