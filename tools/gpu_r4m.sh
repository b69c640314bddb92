#!/usr/bin/env bash
# r4: lock-step exact parts (GPD_EXACT_LOCK=1): bitwise test first (short timeout: a barrier
# mismatch would hang), then C5 exact lock vs default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "lock_step" --timeout 60 --timeout-method thread > $O/tests_lock.log 2>&1 || { tail -40 $O/tests_lock.log; exit 1; }
tail -1 $O/tests_lock.log
for r in 1 2; do
for lk in 1 0; do
  GPD_EXACT_LOCK=$lk timeout -k 10 150 python tools/faint_time.py --method exact --reps 2 > $O/c5_lock$lk$r.json 2>$O/c5_lock$lk$r.err || { tail -20 $O/c5_lock$lk$r.err; exit 1; }
  echo "C5 exact lock=$lk"; cat $O/c5_lock$lk$r.json
done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards.py tests/test_gpu_faint_stats.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
