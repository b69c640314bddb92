#!/usr/bin/env bash
# r5: where the harmonic fit's time goes — NEWUOA phase split (diagnostics variant, GPD_LIB=fdiag)
# and SQ counters of k_fit_harmonic for a lone-series batch (P = 32) and the C4 rank (12500).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5h}
mkdir -p $O
GPD_LIB=fdiag timeout -k 10 180 python tools/fit_probe.py --pixels 32,12500 --reps 3 --prof > $O/fdiag.jsonl 2> $O/fdiag.err || { tail -20 $O/fdiag.err; exit 1; }
grep fit_prof $O/fdiag.err
export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS"
for P in 32 12500; do
  for pass in A B; do
    case $pass in A) C=$PA ;; B) C=$PB ;; esac
    ( cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex k_fit_harmonic -f csv -d "$R/$O/pmc_${P}_$pass" -o pmc -- \
        python3 "$R/tools/fit_probe.py" --pixels $P --reps 1 > "$R/$O/pmc_${P}_$pass.json" 2>&1 ) || { echo "pmc $P $pass failed"; tail -5 "$R/$O/pmc_${P}_$pass.json"; exit 1; }
  done
done
echo done
