# C5-continuous A/B: LDS-DMA tile fills (default) vs register-staged fills (DCOR_TILED_VARIANT=3),
# the 768-thread variant, timing-only ablations (1 no perm loads, 15 no memory phases), then the
# tiled-kernel tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
run() {  # name, switches...
  local n=$1; shift
  local args=()
  for v in "$@"; do args+=(--variant "$v"); done
  timeout -k 10 200 python -u bench_configs.py --only C5c "${args[@]}" > $O/c5c_$n.jsonl 2> $O/c5c_$n.err || return $?
  python3 -c "import json; d=json.loads(open('$O/c5c_$n.jsonl').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['reps_per_s'], round(d['hbm_frac'], 3))"
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hrs.py tests/test_gpu_variants.py > $O/t_hrs.log 2>&1; rc=$?; tail -2 $O/t_hrs.log; [ $rc -ne 0 ] && exit $rc
run dma || exit $?
run nodma DCOR_TILED_VARIANT=3 || exit $?
run dma_b || exit $?
run nodma_b DCOR_TILED_VARIANT=3 || exit $?
run v768 DCOR_TILED_VARIANT=2 || exit $?
for v in 1 15; do
  DCOR_LIB=$PWD/distributed-correlation_amd/dcor/libdcor_abl$v.so run abl$v || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5c_dma -o run -- python3 bench_configs.py --only C5c > $O/prof_c5c_dma.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r06/prof_c5c_dma/run_kernel_stats.csv')):
    if 'premat' in r['Name']: print(r['Name'].split('(')[0][:60], round(float(r['AverageNs'])/1e3, 1))
PY
