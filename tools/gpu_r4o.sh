#!/usr/bin/env bash
# r4: one exposure at G = 8 with plain (temporal) loads of the streamed arrays (GPD_LIB=tnt:
# the one-wave-per-SIMD exact instances built with -DGPD_EXACT_NT=0) vs non-temporal (release).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4o}
mkdir -p $O
for r in 1 2 3; do
for lib in "" tnt; do
  GPD_LIB=$lib timeout -k 10 120 python tools/c2_offsets_timing.py --g8 > $O/c2_$lib$r.jsonl 2> $O/c2_$lib$r.err || { tail -20 $O/c2_$lib$r.err; exit 1; }
  echo "lib=$lib $(grep exact $O/c2_$lib$r.jsonl | python -c 'import sys,json; print([json.loads(l)["kernels_ms"]["fit_exact"] for l in sys.stdin])')"
done
done
