# Code-pair records (packed fma + unorm16) and select-free pass-1 sums: monotonicity check of the
# conversion, every GPU test, the default bench line.  Outputs under gpurun_out/code/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/code
mkdir -p $O
timeout -k 10 60 ./scripts/ubench_pknorm > $O/pknorm.log 2>&1; rc=$?; cat $O/pknorm.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
