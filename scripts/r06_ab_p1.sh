# Headline: pass-1 LDS padding (3 pass-1 workgroups per CU, a pass-2 workgroup beside them).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
for i in 1 2; do
for pad in 0 4096 12288; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --variant DCOR_P1_LDSPAD=$pad > $O/p1pad_$pad.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/p1pad_$pad.log').read().strip().splitlines()[-1]); print('pad $pad', round(d['value']), round(d['ms_per_step'], 4))"
done
done
