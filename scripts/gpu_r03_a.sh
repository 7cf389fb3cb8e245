# Round 3: the grid engine rework (device-expanded items, bounded passes, persistent workers,
# batched RCCL path) and the new C4 / R-table tests, then the reference grids (VG, SG) timed and
# kernel-traced.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_dist.py tests/test_gpu_c4.py \
  tests/test_gpu_rsurface.py tests/test_tables.py tests/test_gpu_launch_shape.py \
  -x -v --timeout 300 --timeout-method thread > $O/r03a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/r03a_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench_configs.py --only VG,SG > $O/r03a_cfg.jsonl 2> $O/r03a_cfg.err || exit $?
cat $O/r03a_cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03a_prof -o run -- python3 bench_configs.py --only VG,SG > $O/r03a_prof.log 2>&1 || exit $?
f=$(find $O/r03a_prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -24
