# Round 3 iteration: GPU tests (DESEL: pytest -k filter to skip), serial headline trace, bench line, config lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${DESEL:+-k "$DESEL"} > $O/it_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/it_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TAG=${TAG:-ser} bash scripts/gpu_r03_serial.sh || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/it_bench.log 2>&1 || exit $?
tail -1 $O/it_bench.log | cut -c1-200
timeout -k 10 600 python -u bench_configs.py --only ${CFGS:-C2,VG,SG,C5,C5f,S} > $O/it_configs.jsonl 2> $O/it_configs.err || exit $?
python -c "
import json
for l in open('$O/it_configs.jsonl'):
    d = json.loads(l); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print(d['config'], '%.3g' % v, 'frac', d.get('roofline_frac', d.get('hbm_frac')))
"
