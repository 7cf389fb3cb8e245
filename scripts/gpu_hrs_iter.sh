# HRS iteration: the HRS GPU tests, then the C5 config lines (coded, continuous, fused, fused continuous).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hrs
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hrs.py tests/test_gpu_more.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hrs or shared_panel or tiled" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench_configs.py --only ${1:-C5,C5c,C5f,C5fc} > $O/configs.jsonl 2> $O/configs.err || exit $?
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print(d['config'], '%.3g reps/s' % d['reps_per_s'], d.get('hbm_frac',''))"
