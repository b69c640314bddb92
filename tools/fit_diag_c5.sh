set -o pipefail
mkdir -p gpurun_out/fdiag
GPD_LIB=fdiag GPD_OPTS=fit_prof=1 timeout -k 10 120 python tools/faint_time.py --reps 2 > gpurun_out/fdiag/c5.json 2> gpurun_out/fdiag/c5.err || exit 1
GPD_LIB=fdiag timeout -k 10 120 python tools/fit_probe.py --pixels 4096 --reps 2 --prof > gpurun_out/fdiag/p4096.json 2> gpurun_out/fdiag/p4096.err || exit 1
grep "fit_prof" gpurun_out/fdiag/c5.err | tail -3; grep fit_prof gpurun_out/fdiag/p4096.err | tail -3
