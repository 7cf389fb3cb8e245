# Kernel-trace stats of config lines: gpu_quick_prof.sh C3 VG ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qp
mkdir -p $O
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- python3 bench_configs.py --only $c --c3-reps 512 > $O/$c.log 2>&1 || exit $?
  f=$(find $O/$c -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('$c', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3), r['Percentage'])
" | head -8
done
