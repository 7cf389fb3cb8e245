# A/B of library builds: headline bench (x2) and config lines per build: gpu_lib_ab.sh CFGS lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
C=$1; shift
for l in "$@"; do
  L=$PWD/distributed-correlation_amd/dcor/$l
  for i in 1 2; do
    DCOR_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/ab_b_$l.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/ab_b_$l.log').read().strip().splitlines()[-1]); print('$l bench', round(d['value']), d['ms_per_step'])"
  done
  DCOR_LIB=$L DCOR_SIGN_PIPELINE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_p_$l -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/ab_p_$l.log 2>&1 || exit $?
  f=$(find $O/ab_p_$l -name '*kernel_stats.csv' | head -1); grep pass2 "$f" | cut -d, -f1-4
  if [ -n "$C" ] && [ "$C" != "-" ]; then
    DCOR_LIB=$L timeout -k 10 300 python -u bench_configs.py --only $C > $O/ab_c_$l.jsonl 2> $O/ab_c_$l.err || exit $?
    python -c "
import json
for x in open('$O/ab_c_$l.jsonl'):
    d = json.loads(x); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print('$l', d['config'], '%.4g' % v)
"
  fi
done
