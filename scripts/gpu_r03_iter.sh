# Round 3 iteration: every GPU test, the headline bench line (no CPU leg), the sign-family config lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/it_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/it_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/it_bench.log 2>&1 || exit $?
tail -1 $O/it_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/it_bench2.log 2>&1 || exit $?
tail -1 $O/it_bench2.log | cut -c1-200
timeout -k 10 600 python -u bench_configs.py --only ${CFGS:-C1,C2,C3,C4,VG,S} > $O/it_configs.jsonl 2> $O/it_configs.err || exit $?
python -c "
import json
for l in open('$O/it_configs.jsonl'):
    d = json.loads(l); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print(d['config'], '%.3g' % v, 'frac', d.get('roofline_frac', d.get('hbm_frac')))
"
