# Tiled-kernel iteration: its parity tests, then C5c for every variant and the L2-gather kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/it
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hrs.py tests/test_gpu_more.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tiled or shared_panel or fused_equals" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
run() {  # name, env...
  local N=$1; shift
  env "$@" timeout -k 10 300 python -u bench_configs.py --only C5c > $O/$N.jsonl 2> $O/$N.err || return $?
  python3 -c "import json; d=json.loads(open('$O/$N.jsonl').read().splitlines()[-1]); print('$N', round(d['seconds']*1e6), 'us', round(d['hbm_frac'], 3))"
}
for V in 0 1; do run v$V DCOR_TILED_VARIANT=$V || exit $?; done
run l2 DCOR_TILED=0 || exit $?
