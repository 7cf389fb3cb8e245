# Round 3: every GPU test, smoke, the bench line, every config line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r03f_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/r03f_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03f_smoke.log 2>&1 || exit $?
tail -1 $O/r03f_smoke.log
timeout -k 10 400 python -u bench.py > $O/r03f_bench.log 2>&1 || exit $?
tail -1 $O/r03f_bench.log | cut -c1-600
timeout -k 10 600 python -u bench_configs.py > $O/r03f_configs.jsonl 2> $O/r03f_configs.err || exit $?
python -c "
import json
for l in open('$O/r03f_configs.jsonl'):
    d = json.loads(l); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print(d['config'], '%.3g' % v, 'frac', d.get('roofline_frac', d.get('hbm_frac')))
"
