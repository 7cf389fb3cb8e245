# GPU: parity tests + headline bench (+ regen A/B).  Stops at the first fault/timeout.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
DCOR_SIGN_KERNEL=regen timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > $O/bench_regen.log 2>&1 || exit $?
tail -1 $O/bench_regen.log
