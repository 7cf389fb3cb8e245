# After a reduction change: every -m gpu test, then the headline and config lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/t_all.log 2>&1; rc=$?; tail -3 $O/t_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_ws.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('$O/bench_ws.log').read().strip().splitlines()[-1]); print('headline', round(d['value']), d['roofline']['issue']['ms'])"
timeout -k 10 400 python -u bench_configs.py --only C5,C5c,VG,SG,C2,C5f,S,C1 > $O/cfg_ws.jsonl 2> $O/cfg_ws.err || exit $?
python3 -c "
import json
for x in open('$O/cfg_ws.jsonl'):
    d = json.loads(x); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print(d['config'], '%.4g' % v, d.get('hbm_frac', ''))
"
