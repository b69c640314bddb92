#!/usr/bin/env bash
# A/B (r6): the C3 step with the moment pass on fewer CUs (option mom_cus) and with pipelined
# cohorts whose fits run on CUs reserved per XCD (options cohorts, fit_cus) — step time and the
# records' hash (they must equal the default's).  → gpurun_out/ab_fit_cus/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/ab_fit_cus
mkdir -p "$OUT"
cd "$R"
run() {
  # bench.py with the options applied first (process-wide); torch first, so that the library
  # binds the HIP runtime torch loaded (loading the library first brings in a second one)
  GPD_OPTS="$1" timeout -k 10 150 python -c "import sys, runpy, torch, gpdemod_loader; gpdemod_loader.load().options_from_env(); \
sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('bench.py', run_name='__main__')" \
      --steps 10 --warmup 2 --no-cpu --no-f64 --no-c4 --no-c5 --no-c2 \
      --dump-records "$OUT/rec.npy" > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; return 1; }
  sleep 3  # let the previous process's 200 GB of device memory go back
  python - "$1" "$OUT" <<'PY'
import hashlib, json, sys
import numpy as np
o = json.loads(open(sys.argv[2] + "/b.json").read().strip().splitlines()[-1])
r = np.load(sys.argv[2] + "/rec.npy")
print(json.dumps({"opts": sys.argv[1], "ms": round(o["ms_per_step"], 3), "k": o.get("kernels_ms"),
                  "records_sha": hashlib.sha256(r.tobytes()).hexdigest()[:16]}))
PY
}
OPTS=${AB_OPTS:-"mom_cus=240|mom_cus=224|cohorts=8|cohorts=8,fit_cus=1|cohorts=8,fit_cus=2|cohorts=4,fit_cus=2|cohorts=16,fit_cus=2"}
IFS='|' read -ra LIST <<< "|$OPTS"
for rep in 1 2; do
  for o in "${LIST[@]}"; do
    run "$o" >> "$OUT/ab.jsonl" || exit 1
  done
done
cat "$OUT/ab.jsonl"
