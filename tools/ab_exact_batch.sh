set -o pipefail
for lib in ${LIBS:-"" u2 ur8}; do
  for m in exact fp32; do
    GPD_LIB=$lib timeout -k 10 200 python tools/faint_time.py --method $m --reps 2 | sed "s/^/lib=$lib /" || exit 1
  done
done
