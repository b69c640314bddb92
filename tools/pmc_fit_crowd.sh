#!/usr/bin/env bash
# Why fit waves slow down when several share a CU: SQ counters of k_fit_harmonic for single-lane
# waves at one wave per CU (256 series) and four per CU (1024 series).  Separate PMC passes, each
# within the gfx950 slot limits (8 SQ, 2 GRBM), never combined with tracing.  → gpurun_out/pmc_fit_crowd/
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_fit_crowd
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
PC="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"
PB="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for P in 256 1024; do
  for pass in ${PASSES:-A B C}; do
    case $pass in A) C=$PA ;; B) C=$PB ;; C) C=$PC ;; esac
    for c in $C; do grep -q "$c" "$OUT/counters.txt" || { echo "missing counter $c"; exit 1; }; done
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex k_fit_harmonic -f csv -d "$OUT/p${P}_$pass" -o pmc -- \
        python3 "$R/tools/fit_lanes_sweep.py" --pixels $P --lanes 1 --reps 2 > "$OUT/p${P}_$pass.json" 2>&1 || exit 1
  done
done
find "$OUT" -name "*.csv" | sort
