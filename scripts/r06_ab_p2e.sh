# Small-cell grids: p2e wave kernels with the global log table (default, 4 workgroups per CU) vs the
# LDS copy (DCOR_P2E_LDS_LT build); then the tests that run these kernels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
for i in 1 2; do
for l in libdcor.so libdcor_ldslt.so; do
  DCOR_LIB=$PWD/distributed-correlation_amd/dcor/$l timeout -k 10 300 python -u bench_configs.py --only C1,C2,VG > $O/p2e_$l.jsonl 2> $O/p2e_$l.err || exit $?
  python3 -c "
import json
for x in open('$O/p2e_$l.jsonl'):
    d = json.loads(x); print('$l', d['config'], '%.4g' % d['reps_per_s'])
"
done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_grid.py tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_fuzz.py tests/test_gpu_launch_shape.py > $O/t_p2e.log 2>&1; rc=$?; tail -2 $O/t_p2e.log; exit $rc
