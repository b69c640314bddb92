#!/usr/bin/env bash
# r5: C3 fit shape sweep (one and two lanes per series, series per wave, waves per workgroup).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 500 python tools/fit_probe.py --pixels 100000 --lps 1 --lanes 40,44,49,56,64 --wpb 1,2,4 --reps 2 > $O/sweep_1e5.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
timeout -k 10 300 python tools/fit_probe.py --pixels 100000 --lps 2 --lanes 22,25,32 --wpb 1,4 --reps 2 >> $O/sweep_1e5.jsonl 2>> $O/s.err || { tail -20 $O/s.err; exit 1; }
python - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/r5o/sweep_1e5.jsonl")]
rows.sort(key=lambda d: d["kernels_ms"]["fit_harmonic"])
for d in rows: print(d["fit_lps"], d["fit_lanes"], d["fit_wpb"], d["kernels_ms"]["fit_harmonic"], d["records_sha"])
PY
