# GPU tests on a candidate build (DCOR_LIB), then an A/B of library builds:
# gpu_r03_ab3.sh CANDIDATE CFGS lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab3
mkdir -p $O
CAND=$1; shift
DCOR_LIB=$PWD/distributed-correlation_amd/dcor/$CAND timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest ($CAND) rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_lib_ab.sh "$@"
