#!/usr/bin/env bash
set -euo pipefail
R=${GRAFT_REPO_ROOT}
OUT=$R/gpurun_out/pmc_clock
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
C="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY"
for v in c64 c32 noload; do
  args="--steps 1 --warmup 0 --no-cpu"
  envset=""
  if [ $v = c32 ]; then args="$args --storage c32"; fi
  if [ $v = noload ]; then export GPD_MOMENTS=ws_noload; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_moments -f csv -d $OUT/$v -o pmc -- python3 $R/bench.py $args > $OUT/$v.json
  unset GPD_MOMENTS
done
find $OUT -name "*.csv" | sort
