# The round-end gate as the driver runs it (every -m gpu test, smoke), then bench.py with its
# defaults (CPU baseline included) -> gpurun_out/r06_bench_headline.jsonl.
set -o pipefail
export TMPDIR=/tmp
bash scripts/check.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r06_bench.log 2>&1; rc=$?
tail -1 gpurun_out/r06_bench.log > gpurun_out/r06_bench_headline.jsonl
tail -1 gpurun_out/r06_bench.log | cut -c1-300; exit $rc
