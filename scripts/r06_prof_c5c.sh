# Counters of the C5-continuous kernels and of the serial headline on the current tree.
set -o pipefail
export TMPDIR=/tmp
bash scripts/prof.sh r06w_c5c trace,sq,mix,lds -- bench_configs.py --only C5c || exit $?
SERIAL=1 bash scripts/prof.sh r06w_serial trace,sq,mix -- bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-ceilings || exit $?
