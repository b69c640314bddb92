#!/usr/bin/env bash
# r5: where the C2 host-buffer call's time goes (gpd_demodulateall), the C5 faint step with the
# multi-lane fit, and SQ counters of the faint vs plain moment kernel on 4096 × 1e5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5f}
mkdir -p $O
timeout -k 10 120 python tools/c2_host.py 7 > $O/c2_host.json 2> $O/c2_host.err || { tail -20 $O/c2_host.err; exit 1; }
cat $O/c2_host.json; grep host_prof $O/c2_host.err
timeout -k 10 120 python tools/faint_time.py --reps 5 > $O/c5_harm.json 2> $O/c5_harm.err || { tail -20 $O/c5_harm.err; exit 1; }
cat $O/c5_harm.json
timeout -k 10 400 bash tools/pmc_moments_sq.sh > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 1; }
tail -3 $O/pmc_sq.log
