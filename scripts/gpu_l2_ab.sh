# GPU tests, then the C5-continuous line under each uncoded-panel kernel variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 0 1 2 3; do
  DCOR_L2_VARIANT=$v timeout -k 10 300 python -u bench_configs.py --only C5c,C5 > $O/l2_$v.jsonl 2> $O/l2_$v.err || exit $?
  python -c "
import json
for l in open('$O/l2_$v.jsonl'):
    d=json.loads(l); print('variant $v', d['config'], round(d['reps_per_s']), round(d['hbm_frac'],3), d['kernel'])"
done
