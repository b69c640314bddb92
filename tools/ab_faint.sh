#!/usr/bin/env bash
# A/B of the faint statistics (GPD_LIB variants): C5 harmonic step, per-kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
for rep in 1 2; do
  for lib in "" "$@"; do
    GPD_LIB=$lib timeout -k 10 100 python tools/faint_time.py --reps 5 | sed "s/^/lib=$lib /" || exit 1
  done
done
