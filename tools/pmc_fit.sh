#!/usr/bin/env bash
# Instruction-cache and issue counters of k_fit_harmonic (one PMC pass per counter group).
# Usage: tools/pmc_fit.sh <tag> [bench args...]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmcfit_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -o -E "SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_WAIT_INST_ANY|SQ_INSTS_VALU\b" "$OUT/counters.txt" | sort -u > "$OUT/names.txt"
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_IFETCH" \
         "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
         "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex k_fit_harmonic -f csv -d "$OUT/p$i" -o pmc -- \
      python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  echo "pass $i rc=$?"
done
