#!/usr/bin/env bash
# A/B of library builds on one box, interleaved rounds (box-to-box spread is ~6 %, so only
# same-box comparisons count).  Usage: tools/ab_bench.sh <tag> <rounds> <bench args> -- <variant>...
# A variant is "name:GPD_LIB=x" ("base:" = the release library); GPD_LIB=old loads
# libgpdemod_old.so.  The library reads no environment variable and bench.py applies no options,
# so a build variant (build.py --variant) is the only knob here.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ROUNDS=$2; shift 2
ARGS=()
while [ "$1" != "--" ]; do ARGS+=("$1"); shift; done
shift
OUT=$R/gpurun_out/ab_$TAG.jsonl
mkdir -p "$R/gpurun_out"; : > "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    line=$(env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python3 "$R/bench.py" "${ARGS[@]}" | tail -1)
    echo "{\"variant\": \"$name\", \"round\": $r, \"bench\": $line}" >> "$OUT"
    echo "$name r$r: $(echo "$line" | python3 -c 'import json,sys; j=json.load(sys.stdin); print(round(j["ms_per_step"],3), j["kernels_ms"])')"
  done
done
