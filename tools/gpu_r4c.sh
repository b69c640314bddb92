#!/usr/bin/env bash
# r4: wave-level split of the phase-scheduled fit (diag build): C4 rank, one exposure-sized batch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r4c
for p in 12500 4096 1024; do
  GPD_LIB=diag GPD_FIT_PROF=1 timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --no-f64 --no-c4 --no-c5 --pixels $p > gpurun_out/r4c/fitprof_$p.json 2> gpurun_out/r4c/fitprof_$p.err || exit 1
  echo "P=$p"; grep fit_prof gpurun_out/r4c/fitprof_$p.err | tail -4
done
