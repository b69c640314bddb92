#!/usr/bin/env bash
# r5: fit-shape sweep after the NEWUOB state walk (divergence cost changed): C4 rank (12500),
# 4096 (C5 shape), C3 (1e5).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5j}
mkdir -p $O
timeout -k 10 300 python tools/fit_probe.py --pixels 12500 --lps 2,4,8 --lanes 8,10,12,13,16 --wpb 1,4 --reps 3 > $O/sweep_12500.jsonl 2> $O/s1.err || { tail -20 $O/s1.err; exit 1; }
timeout -k 10 300 python tools/fit_probe.py --pixels 4096 --lps 4,8 --lanes 2,3,4,6,8 --wpb 1,2,4 --reps 3 > $O/sweep_4096.jsonl 2> $O/s2.err || { tail -20 $O/s2.err; exit 1; }
timeout -k 10 400 python tools/fit_probe.py --pixels 100000 --lps 1,2 --lanes 25,32,40,49,56,64 --wpb 1,4 --reps 2 > $O/sweep_1e5.jsonl 2> $O/s3.err || { tail -20 $O/s3.err; exit 1; }
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r5j/sweep_*.jsonl")):
    rows=[json.loads(l) for l in open(f)]
    rows.sort(key=lambda d: d["kernels_ms"]["fit_harmonic"])
    print(f, [(d["fit_lps"], d["fit_lanes"], d["fit_wpb"], d["kernels_ms"]["fit_harmonic"]) for d in rows[:6]], len(set(d["records_sha"] for d in rows)))
PY
GPD_LIB=fdiag timeout -k 10 180 python tools/fit_probe.py --pixels 32,4096,12500,100000 --reps 2 --prof > $O/fdiag.jsonl 2> $O/fdiag.err || { tail -20 $O/fdiag.err; exit 1; }
grep "fit_prof per wave" $O/fdiag.err
