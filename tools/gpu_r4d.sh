#!/usr/bin/env bash
# r4: fit scheduler variants (greedy/fixed order × switch/sequential glue) against run():
# C4 rank and C5 fit time; C3 for the release and run(); diag phase split.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r4d
mkdir -p $O
for lib in "" seqglue fixed tree treenosched nosched; do
  GPD_LIB=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --no-f64 --no-c4 --no-c5 --pixels 12500 \
    | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','shape':'c4rank','ms':round(j['ms_per_step'],3),'fit':j['kernels_ms']['fit_harmonic']}))" >> $O/ab.jsonl || exit 1
  GPD_LIB=$lib timeout -k 10 100 python tools/faint_time.py --reps 5 \
    | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','shape':'c5','wall':j['wall_ms'],'fit':j['kernels_ms']['fit_harmonic']}))" >> $O/ab.jsonl || exit 1
done
cat $O/ab.jsonl
for p in 12500 1024; do
  GPD_LIB=diag GPD_FIT_PROF=1 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --no-f64 --no-c4 --no-c5 --pixels $p > $O/fitprof_$p.json 2> $O/fitprof_$p.err || exit 1
  echo "P=$p"; grep fit_prof $O/fitprof_$p.err | tail -4
done
