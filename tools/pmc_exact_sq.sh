#!/usr/bin/env bash
# r4: SQ counters (instruction mix, waits) of k_fit_exact for C2 exact (one exposure, G = 8) and
# C5 exact (4096 series, G = 1), one PMC pass each.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_exact_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_fit_exact -f csv -d "$OUT/c2" -o pmc -- \
    python3 "$R/tools/c2_offsets_timing.py" --g8 > "$OUT/c2.jsonl"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_fit_exact -f csv -d "$OUT/c5" -o pmc -- \
    python3 "$R/tools/faint_time.py" --method exact --reps 1 > "$OUT/c5.json"
find "$OUT" -name "*.csv" | sort
