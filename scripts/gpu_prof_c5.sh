# C5 refresh: configs (C5, C5c, C5e) + kernel-trace stats + one FETCH_SIZE PMC pass.
# Usage: bash scripts/gpu_prof_c5.sh   (outputs under gpurun_out/c5r/)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5r
mkdir -p $O
timeout -k 10 300 python -u bench_configs.py --only C5,C5c,C5e > $O/configs.jsonl 2> $O/configs.err || exit $?
cat $O/configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench_configs.py --only C5,C5e > $O/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench_configs.py --only C5 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench_configs.py --only C5e > $O/write.log 2>&1 || exit $?
echo done
