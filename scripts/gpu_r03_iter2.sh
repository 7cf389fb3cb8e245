# Round 3 iteration: every GPU test, the serial-chunk kernel trace of the headline, the bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/it_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/it_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
TAG=${TAG:-ser} bash scripts/gpu_r03_serial.sh || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/it_bench.log 2>&1 || exit $?
tail -1 $O/it_bench.log | cut -c1-300
