# A/B of config lines across library builds: gpu_cfg_ab.sh CFGS lib1 lib2 ... (lib = dcor/libdcor*.so name)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
C=$1; shift
for rep in 1 2; do
for l in "$@"; do
  DCOR_LIB=$PWD/distributed-correlation_amd/dcor/$l timeout -k 10 300 python -u bench_configs.py --only $C > $O/ab_$l.jsonl 2> $O/ab_$l.err || exit $?
  python -c "
import json
for x in open('$O/ab_$l.jsonl'):
    d = json.loads(x); v = d.get('reps_per_s', d.get('gpu_reps_per_s', d.get('runs_per_s')))
    print('$l', d['config'], '%.4g' % v)
"
done
done
