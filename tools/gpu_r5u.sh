#!/usr/bin/env bash
# r5: Bessel recurrence with one fma per step — fit times (records change by the recurrence's
# rounding: new hashes), the GPU suite (harmonic parity within its tolerances).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5u
mkdir -p $O
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 5 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
GPD_LIB=fdiag timeout -k 10 180 python tools/fit_probe.py --pixels 32,12500 --reps 2 --prof > $O/fdiag.jsonl 2> $O/fdiag.err || { tail -20 $O/fdiag.err; exit 1; }
grep "fit_prof per" $O/fdiag.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
