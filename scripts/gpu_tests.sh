# A subset of the -m gpu tests (pytest -k expression or files), one process, each bounded.
#   bash scripts/gpu_tests.sh "<pytest args>"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread $1 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log; exit $rc
