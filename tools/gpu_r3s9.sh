#!/usr/bin/env bash
# Late round 3: whole GPU suite (alignment test included), smoke, C5 timing, default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_suite_s9.log 2>&1 || { tail -40 gpurun_out/gpu_suite_s9.log; exit 1; }
tail -1 gpurun_out/gpu_suite_s9.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 100 python tools/faint_time.py --reps 5 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_s9.json 2> gpurun_out/bench_s9.err || { tail -20 gpurun_out/bench_s9.err; exit 1; }
python -c "import json; j=json.load(open('gpurun_out/bench_s9.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j.get('kernels_ms'))"
