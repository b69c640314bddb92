#!/usr/bin/env bash
# r5: the harmonic objective out of line with its inputs by value, moments from LDS (fit_mcache)
# — records must keep their hashes (32 7e6072a976bd62d9, 4096 d4d6d0c45ad2d127, 12500
# 68315e794012bda1, 1e5 bdf82ee520073785); A/B fit_mcache 0; NEWUOA split; GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5k}
mkdir -p $O
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 5 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
timeout -k 10 60 ./tools/probes/sqrt_ulp > $O/sqrt_ulp.json && cat $O/sqrt_ulp.json
GPD_OPTS=fit_mcache=0 timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500 --reps 5 > $O/probe_nomc.jsonl 2> $O/probe_nomc.err || { tail -20 $O/probe_nomc.err; exit 1; }
cat $O/probe_nomc.jsonl
GPD_LIB=fdiag timeout -k 10 180 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 2 --prof > $O/fdiag.jsonl 2> $O/fdiag.err || { tail -20 $O/fdiag.err; exit 1; }
grep "fit_prof" $O/fdiag.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
