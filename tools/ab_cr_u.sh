#!/bin/bash
# Same-box A/B of exact-path batch sizes on the C2 exposure (G = 8): libgpdemod_<v>.so variants
# built with -DGPD_CR_U=n (first passes) or -DGPD_CR_UR=n (residual pass), plus GPD_FIT_PROF's
# per-phase cycle split for the default build.  Usage: tools/ab_cr_u.sh [variant ...]
set -e
mkdir -p gpurun_out
for L in "" "$@"; do
  for m in "" --mjd; do
    GPD_LIB=$L timeout -k 10 120 python tools/c2_offsets_timing.py --g8 $m >> gpurun_out/cu.log 2>&1
  done
done
GPD_FIT_PROF=1 timeout -k 10 120 python tools/c2_offsets_timing.py --g8 --mjd >> gpurun_out/cu.log 2>&1
