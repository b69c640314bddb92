#!/usr/bin/env bash
# State-split faint moments (serial statistics by default): faint tests, C5 step timing
# (default and GPD_FAINT_SIDE=1), full GPU suite, default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "faint or shards or c32 or states or cohort" > gpurun_out/gpu_faint_s4.log 2>&1 || { tail -40 gpurun_out/gpu_faint_s4.log; exit 1; }
tail -1 gpurun_out/gpu_faint_s4.log
for side in 0 1; do
  GPD_FAINT_SIDE=$side timeout -k 10 100 python tools/faint_time.py --reps 5 | sed "s/^/side=$side /" || exit 1
done
timeout -k 10 100 python tools/faint_time.py --reps 5 --c32 | sed "s/^/c32 /" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_suite_s4.log 2>&1 || { tail -40 gpurun_out/gpu_suite_s4.log; exit 1; }
tail -1 gpurun_out/gpu_suite_s4.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_s4.json 2> gpurun_out/bench_s4.err || { tail -20 gpurun_out/bench_s4.err; exit 1; }
python -c "import json; j=json.load(open('gpurun_out/bench_s4.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j.get('kernels_ms'))"
