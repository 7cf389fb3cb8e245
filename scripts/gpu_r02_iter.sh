# Round-2 iteration call: the GPU test suite, two headline bench runs, chosen config lines.
# Usage: bash scripts/gpu_r02_iter.sh [config ids, default C5,C5c,C5f,C5fc]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel_ms_avg'])"
done
timeout -k 10 600 python -u bench_configs.py --only ${1:-C5,C5c,C5f,C5fc} > $O/configs_iter.jsonl 2> $O/configs_iter.err || exit $?
cat $O/configs_iter.jsonl | cut -c1-300
