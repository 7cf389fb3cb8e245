# Kernel stats of the C1 line per library build: gpu_c1_ab.sh lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c1ab
mkdir -p $O
for l in "$@"; do
  L=$PWD/distributed-correlation_amd/dcor/$l
  DCOR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$l -o run -- python3 bench_configs.py --only C1 > $O/c1_$l.log 2>&1 || exit $?
  f=$(find $O/p_$l -name '*kernel_stats.csv' | head -1); echo "== $l"; cut -d, -f1-5 "$f" | head -8
done
