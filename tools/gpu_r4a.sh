#!/usr/bin/env bash
# r4: parallel k_prepare / k_faint_defer scans — whole GPU suite, smoke, C5 + C2 timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gpu_suite_r4a.log 2>&1 || { tail -40 gpurun_out/gpu_suite_r4a.log; exit 1; }
tail -1 gpurun_out/gpu_suite_r4a.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 100 python tools/faint_time.py --reps 5 > gpurun_out/r4a_c5.json || exit 1
cat gpurun_out/r4a_c5.json
timeout -k 10 120 python tools/host_path.py > gpurun_out/r4a_host_path.json 2> gpurun_out/r4a_host_path.err || { tail -20 gpurun_out/r4a_host_path.err; exit 1; }
cat gpurun_out/r4a_host_path.json
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err || { tail -30 gpurun_out/bench_r4a.err; exit 1; }
python -c "import json; j=json.load(open('gpurun_out/bench_r4a.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['build_id']); print(json.dumps(j['c5_faint'])); print(json.dumps(j['cpu_baseline']['parity'].get('reference_ceiling'))); print(json.dumps(j['cpu_baseline']['c1_one_diode']))"
