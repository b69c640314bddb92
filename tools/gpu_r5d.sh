#!/usr/bin/env bash
# r5: multi-lane harmonic fit (phase 1: canonical objective + split angle searches, the library
# kept as libgpdemod_ph1.so; phase 2: + grid / initial points / π-flip evaluated in parallel)
# and gpd_demodulateall — shape invariance, the new entry point, fit-shape sweep (both phases),
# GPU suite, smoke, bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards.py tests/test_gpu_parity.py -x -q -k "series_per_fit_wave or demodulateall" --timeout 200 --timeout-method thread > $O/new_tests.log 2>&1 || { tail -40 $O/new_tests.log; exit 1; }
tail -1 $O/new_tests.log
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500 --lps 0,1,2,4,8 --wpb 1,4 > $O/fit_probe.jsonl 2> $O/fit_probe.err || { tail -20 $O/fit_probe.err; exit 1; }
GPD_LIB=ph1 timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500 --lps 0,1,2,4,8 --wpb 1,4 > $O/fit_probe_ph1.jsonl 2> $O/fit_probe_ph1.err || { tail -20 $O/fit_probe_ph1.err; exit 1; }
timeout -k 10 120 python tools/fit_probe.py --pixels 12500 --lps 1,2,4 --lanes 13,16,25,32,49 --wpb 1,4 > $O/fit_probe_c4.jsonl 2> $O/fit_probe_c4.err || { tail -20 $O/fit_probe_c4.err; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --no-c5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['kernels_ms'], j['c4_rank_rehearsal']['kernels_ms'], j['c4_rank_rehearsal']['projected_speedup_at_8_gpus'], j['cpu_baseline']['parity']['within_1e-10'], j['cpu_baseline']['parity']['unexplained'], json.dumps(j['c2_exposure']['cases']))"
