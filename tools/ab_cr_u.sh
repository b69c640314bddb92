set -e
mkdir -p gpurun_out
for L in "" u2 u6 u8; do
  for m in "" --mjd; do
    GPD_LIB=$L timeout -k 10 120 python tools/c2_offsets_timing.py --g8 $m >> gpurun_out/cu.log 2>&1
  done
done
GPD_FIT_PROF=1 timeout -k 10 120 python tools/c2_offsets_timing.py --g8 --mjd >> gpurun_out/cu.log 2>&1
