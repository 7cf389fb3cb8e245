set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench_configs.py --only ${ONLY:-C5} > $O/c5.jsonl 2> $O/c5.err || exit $?
cat $O/c5.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench_configs.py --only ${ONLY:-C5} > $O/prof_c5.log 2>&1 || exit $?
f=$(find $O/prof_c5 -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -12
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_c5_fetch -o run -- python3 bench_configs.py --only ${ONLY:-C5} > $O/prof_c5_fetch.log 2>&1 || exit $?
echo fetch-done
