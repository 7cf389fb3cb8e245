# rocprofv3 kernel trace of the R-stream lines (R1, RG, RH).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/rsprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench_configs.py --only R1,RG,RH > $O/trace.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -3
