# Kernel-trace profile of bench_configs.py configs: ONLY=C2,C5 bash scripts/gpu_prof_configs.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
T=${TAG:-cfg}
timeout -k 10 300 python -u bench_configs.py --only ${ONLY:-C5} > $O/$T.jsonl 2> $O/$T.err || exit $?
cat $O/$T.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 bench_configs.py --only ${ONLY:-C5} > $O/prof_$T.log 2>&1 || exit $?
f=$(find $O/prof_$T -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -14
