set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --reps 2048 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
  echo "bench rc=$?"
  cat gpurun_out/bench.log | tail -5
fi
