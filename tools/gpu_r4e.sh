#!/usr/bin/env bash
# r4: one run() call site in drive_fit (kernel code 19.5 k -> 10.5 k instructions): GPU suite,
# fit time against series per wave (crowding) for the C4 rank, C5 and C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for lanes in auto 25 13; do
  if [ $lanes = auto ]; then unset GPD_FIT_LANES; else export GPD_FIT_LANES=$lanes; fi
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 --no-c4 --no-c5 --pixels 12500 \
    | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'lanes':'$lanes','shape':'c4rank','ms':round(j['ms_per_step'],3),'fit':j['kernels_ms']['fit_harmonic']}))" >> $O/lanes.jsonl || exit 1
done
for lanes in auto 8 4; do
  if [ $lanes = auto ]; then unset GPD_FIT_LANES; else export GPD_FIT_LANES=$lanes; fi
  timeout -k 10 100 python tools/faint_time.py --reps 5 \
    | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'lanes':'$lanes','shape':'c5','wall':j['wall_ms'],'fit':j['kernels_ms']['fit_harmonic']}))" >> $O/lanes.jsonl || exit 1
done
unset GPD_FIT_LANES
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 --no-c5 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python -c "import json; j=json.load(open('$O/c3.json')); print('c3', j['ms_per_step'], j['kernels_ms'], j['c4_rank_rehearsal'])"
cat $O/lanes.jsonl
