# A/B of engine builds (scripts/build_variant.sh): for each library, the headline bench twice, a
# serial kernel trace (per-pass times) and, optionally, config lines.
#   bash scripts/ab.sh <CFGS|-> libdcor.so libdcor_x.so ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
C=$1; shift
for l in "$@"; do
  L=$PWD/distributed-correlation_amd/dcor/$l
  for i in 1 2; do
    DCOR_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_$l.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/b_$l.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$l bench', round(d['value']), round(d['ms_per_step'], 4), 'issue', r['issue'] and {k: r['issue']['ms'][k] for k in ('pass1', 'pass2', 'epilogue', 'pass1_ceiling', 'pass2_ceiling')})"
  done
  if [ -n "$C" ] && [ "$C" != "-" ]; then
    DCOR_LIB=$L timeout -k 10 600 python -u bench_configs.py --only $C > $O/c_$l.jsonl 2> $O/c_$l.err || exit $?
    python -c "
import json
for x in open('$O/c_$l.jsonl'):
    d = json.loads(x); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print('$l', d['config'], '%.4g' % v)
"
  fi
done
