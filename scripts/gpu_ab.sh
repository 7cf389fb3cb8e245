# A/B of the headline bench under environment variants: gpu_ab.sh "VAR=a" "VAR=b" ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/ab_$i.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('$O/ab_$i.log').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['roofline']['frac'],4), d['roofline']['kernel_ms_avg'])"
done
