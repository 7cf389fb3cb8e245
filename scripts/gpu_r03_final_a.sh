# Round 3 final evidence, part A: every GPU test, smoke(), the default bench line (with the CPU
# baselines), every config line.  Outputs under gpurun_out/final/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 700 python -u bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit $?
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print(d['config'], '%.3g' % v, 'frac', d.get('roofline_frac', d.get('hbm_frac')))
"
