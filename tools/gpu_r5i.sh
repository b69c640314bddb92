#!/usr/bin/env bash
# r5: NEWUOB as an explicit state walk (the fits of a wave meet at the objective) — the fit
# probe's records must keep their hashes (r5 sweeps: 32 7e6072a976bd62d9, 4096
# d4d6d0c45ad2d127, 12500 68315e794012bda1, 1e5 bdf82ee520073785); times; NEWUOA phase split
# (GPD_LIB=fdiag); then the GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5i}
mkdir -p $O
timeout -k 10 240 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 5 > $O/probe.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.jsonl
GPD_LIB=fdiag timeout -k 10 180 python tools/fit_probe.py --pixels 32,12500 --reps 3 --prof > $O/fdiag.jsonl 2> $O/fdiag.err || { tail -20 $O/fdiag.err; exit 1; }
grep fit_prof $O/fdiag.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
