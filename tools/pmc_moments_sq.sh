#!/usr/bin/env bash
# r5: SQ counters of the moment kernel k_moments_ws on the 4096 × 1e5 shape, faint (C5:
# tools/faint_time.py, state-split moments + fused statistics) against non-faint
# (tools/fit_probe.py --pixels 4096), two PMC passes each (≤ 8 SQ + ≤ 2 GRBM counters per pass,
# never combined with tracing).  → gpurun_out/pmc_moments_sq/
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_moments_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
for c in $PA $PB; do grep -q "$c" "$OUT/counters.txt" || { echo "missing counter $c"; exit 1; }; done
for pass in A B; do
  case $pass in A) C=$PA ;; B) C=$PB ;; esac
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_moments_ws -f csv -d "$OUT/faint_$pass" -o pmc -- \
      python3 "$R/tools/faint_time.py" --reps 1 > "$OUT/faint_$pass.json" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_moments_ws -f csv -d "$OUT/plain_$pass" -o pmc -- \
      python3 "$R/tools/fit_probe.py" --pixels 4096 --reps 1 > "$OUT/plain_$pass.json" 2>&1 || exit 1
done
find "$OUT" -name "*.csv" | sort
