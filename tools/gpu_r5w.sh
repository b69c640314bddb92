#!/usr/bin/env bash
# r5: per-role cycle split of the moment kernel (k_moments_ws<6>, diagnostics build) on the
# 4096-series shape — do the consumers wait for the producers?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5w
mkdir -p $O
GPD_LIB=fdiag GPD_OPTS=moments=7 timeout -k 10 120 python tools/fit_probe.py --pixels 4096 --reps 2 > $O/ws_prof.jsonl 2> $O/ws_prof.err || { tail -20 $O/ws_prof.err; exit 1; }
grep ws_prof $O/ws_prof.err | tail -3
