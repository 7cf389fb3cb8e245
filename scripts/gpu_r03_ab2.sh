# GPU tests on the current build, then an A/B of library builds (headline x2, serial pass-2 trace,
# config lines) -- gpu_r03_ab2.sh CFGS lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_lib_ab.sh "$@"
