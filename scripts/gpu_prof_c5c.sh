# C5-continuous kernel trace: tiled kernel (variant ${1:-0}) and the L2-gather kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5c
mkdir -p $O
DCOR_TILED_VARIANT=${1:-0} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tiled -o run -- python3 bench_configs.py --only C5c > $O/tiled.log 2>&1 || exit $?
DCOR_TILED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l2 -o run -- python3 bench_configs.py --only C5c > $O/l2.log 2>&1 || exit $?
for f in $O/tiled $O/l2; do echo "== $f"; cat $(find $f -name '*kernel_stats.csv') | cut -d, -f1-8 | head -12; done
