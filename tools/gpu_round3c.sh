#!/usr/bin/env bash
# round-3 evidence: C5 sweep (with Float32 arithmetic), rocprof trace + PMC of the C3 bench, and
# the default bench line (CPU baseline with the 8-thread C2 timing).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python tools/c5_sweep.py --out gpurun_out/c5_sweep_r3.json > gpurun_out/c5_sweep_r3.log 2>&1 || { tail -20 gpurun_out/c5_sweep_r3.log; exit 1; }
timeout -k 10 900 bash tools/profile.sh r3 > gpurun_out/profile_r3.log 2>&1 || { tail -20 gpurun_out/profile_r3.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_r3.json 2> gpurun_out/bench_r3.err || { tail -20 gpurun_out/bench_r3.err; exit 1; }
python -c "import json; j=json.load(open('gpurun_out/bench_r3.json')); print(j['value'], j['ms_per_step'], j['roofline']['frac'], j['kernels_ms'])"
