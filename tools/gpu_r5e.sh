#!/usr/bin/env bash
# r5: fit shape sweep (lanes per series × series per wave × waves per workgroup) on C2/C5/C4-rank/C3
# batch sizes with the phase-2 library, the phase-1 library's automatic shape for comparison, then
# the GPU suite, smoke and the bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5e}
mkdir -p $O
GPD_LIB=ph1 timeout -k 10 120 python tools/fit_probe.py --pixels 32,4096,12500 > $O/fit_probe_ph1.jsonl 2> $O/fit_probe_ph1.err || { tail -20 $O/fit_probe_ph1.err; exit 1; }
timeout -k 10 200 python tools/fit_probe.py --pixels 32,256 --lps 4,8 --lanes 1,2,4 --wpb 1 > $O/sweep_small.jsonl 2> $O/sweep_small.err || { tail -20 $O/sweep_small.err; exit 1; }
timeout -k 10 200 python tools/fit_probe.py --pixels 4096 --lps 4,8 --lanes 1,2,4,8,16 --wpb 1,2,4 > $O/sweep_4096.jsonl 2> $O/sweep_4096.err || { tail -20 $O/sweep_4096.err; exit 1; }
timeout -k 10 200 python tools/fit_probe.py --pixels 12500 --lps 2,4,8 --lanes 4,8,13,16,32 --wpb 1,2,4 > $O/sweep_12500.jsonl 2> $O/sweep_12500.err || { tail -20 $O/sweep_12500.err; exit 1; }
timeout -k 10 200 python tools/fit_probe.py --pixels 100000 --lps 1,2 --lanes 32,64 --wpb 1,4 --reps 3 > $O/sweep_1e5.jsonl 2> $O/sweep_1e5.err || { tail -20 $O/sweep_1e5.err; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --no-c5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['kernels_ms'], j['c4_rank_rehearsal']['kernels_ms'], j['c4_rank_rehearsal']['projected_speedup_at_8_gpus'], j['cpu_baseline']['parity']['within_1e-10'], j['cpu_baseline']['parity']['unexplained'], json.dumps(j['c2_exposure']['cases']))"
