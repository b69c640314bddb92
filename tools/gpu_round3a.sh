set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_suite.log 2>&1 || { echo SUITE_FAILED; tail -30 gpurun_out/gpu_suite.log; exit 1; }
tail -3 gpurun_out/gpu_suite.log
for L in 64 16 4 1; do GPD_LIB=diag GPD_FIT_PROF=1 GPD_FIT_LANES=$L timeout -k 10 120 python bench.py --steps 1 --warmup 1 --no-cpu --no-f64 --pixels 12500 > gpurun_out/fitlanes_$L.json 2> gpurun_out/fitlanes_$L.err || exit 1; done
timeout -k 10 300 python tools/window_sweep.py > gpurun_out/window_sweep.json 2> gpurun_out/window_sweep.err
