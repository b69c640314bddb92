#!/usr/bin/env bash
# r5: faint moment kernel without spills (one LDS base for the 16 q stores) — parity on the
# faint/demodulateall tests, the C5 faint step, its SQ counters; the C2 host call with the
# pipelined staged output (chunked D2H + pre-touched destination).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out/${TAG:-r5g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "faint or demodulateall or window or shard" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/faint_time.py --reps 5 > $O/c5_harm.json 2> $O/c5_harm.err || { tail -20 $O/c5_harm.err; exit 1; }
cat $O/c5_harm.json
timeout -k 10 120 python tools/c2_host.py 7 > $O/c2_host.json 2> $O/c2_host.err || { tail -20 $O/c2_host.err; exit 1; }
cat $O/c2_host.json; grep host_prof $O/c2_host.err
export TMPDIR=/tmp
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $PA --kernel-include-regex k_moments_ws -f csv -d "$R/$O/pmc_faint_A" -o pmc -- \
      python3 "$R/tools/faint_time.py" --reps 1 > "$R/$O/pmc_faint_A.json" 2>&1 ) || exit 1
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $PB --kernel-include-regex k_moments_ws -f csv -d "$R/$O/pmc_faint_B" -o pmc -- \
      python3 "$R/tools/faint_time.py" --reps 1 > "$R/$O/pmc_faint_B.json" 2>&1 ) || exit 1
echo done
