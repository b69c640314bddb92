#!/usr/bin/env bash
# r5: the multi-lane harmonic fit (canonical objective, split angle searches, fit shapes) —
# GPU suite, smoke, the fit-shape sweep (records must not depend on the shape), the bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards.py -x -q -k "series_per_fit_wave" --timeout 200 --timeout-method thread > $O/shape_test.log 2>&1 || { tail -40 $O/shape_test.log; exit 1; }
tail -1 $O/shape_test.log
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500 --lps 0,1,2,4,8 --wpb 1,4 > $O/fit_probe.jsonl 2> $O/fit_probe.err || { tail -20 $O/fit_probe.err; exit 1; }
timeout -k 10 120 python tools/fit_probe.py --pixels 12500 --lps 1,4 --lanes 13,16,25,49 --wpb 1,4 > $O/fit_probe_c4.jsonl 2> $O/fit_probe_c4.err || { tail -20 $O/fit_probe_c4.err; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --no-c5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['kernels_ms'], j['c4_rank_rehearsal']['kernels_ms'], j['c4_rank_rehearsal']['projected_speedup_at_8_gpus'], j['cpu_baseline']['parity']['within_1e-10'], j['cpu_baseline']['parity']['unexplained'])"
