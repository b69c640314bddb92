#!/usr/bin/env bash
# Cycles / clock / VALU counts of k_moments_ws timing variants (GPD_MOMENTS=...), one PMC pass each.
# Usage: tools/pmc_variants.sh <tag> <variant>...   (variant "ws" = the production kernel)
# The variants live in the diagnostics build only: build it first on the CPU side
#   python gppupildemodulation.jl_amd/build.py --diag     (→ libgpdemod_diag.so, loaded via GPD_LIB=diag)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmcv_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for v in "$@"; do
  GPD_LIB=diag GPD_MOMENTS=$v timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex k_moments -f csv \
      -d "$OUT/$v" -o pmc -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu > "$OUT/$v.json"
done
