#!/usr/bin/env bash
# r4: the default bench line (C3 headline, sustained block, C4 rank rehearsal, C5 harmonic +
# exact, CPU baselines) and a rocprofv3 kernel trace of the C3 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4k}
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['kernels_ms'], j['sustained'], j['c5_faint']['gpu'], j['c5_faint'].get('gpu_exact'))"
bash tools/profile.sh ${TAG:-r4k} > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -3 $O/profile.log
