#!/usr/bin/env bash
# r5 second GPU pass: the pruned library with the options API (suite, smoke), the bench line,
# the exact evaluator with and without its model cache (C5 exact, C2 exact/fitoffsets), and the
# harmonic fit's series-per-wave curve on a C4 rank shard and smaller batches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for mc in 1 0 1 0; do
  GPD_OPTS=exact_mcache=$mc timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 >> $O/c5_exact_mc.jsonl 2>>$O/c5_exact_mc.err || { tail -20 $O/c5_exact_mc.err; exit 1; }
  GPD_OPTS=exact_mcache=$mc timeout -k 10 120 python tools/c2_offsets_timing.py --g8 >> $O/c2_exact_mc.jsonl 2>> $O/c2_exact_mc.err || { tail -20 $O/c2_exact_mc.err; exit 1; }
done
timeout -k 10 200 python tools/fit_probe.py --pixels 32,4096,12500 --lanes 0,1,4,13,16,25,64 > $O/fit_probe.jsonl 2> $O/fit_probe.err || { tail -20 $O/fit_probe.err; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; j=json.load(open('$O/bench.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['kernels_ms'], j['c4_rank_rehearsal']['kernels_ms'], j['c5_faint']['gpu']['ms_per_step'], json.dumps(j['c2_exposure']['cases']))"
