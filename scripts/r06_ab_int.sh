# C5-continuous: replicates per INT workgroup (DCOR_INT_R 4 default, 2, 8), two runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
for i in 1 2; do
for l in libdcor.so libdcor_r8.so libdcor_r2.so; do
  DCOR_LIB=$PWD/distributed-correlation_amd/dcor/$l timeout -k 10 200 python -u bench_configs.py --only C5c > $O/int_$l.jsonl 2> $O/int_$l.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/int_$l.jsonl').read().strip().splitlines()[-1]); print('$l', '%.4g' % d['reps_per_s'], round(d['hbm_frac'], 3))"
done
done
