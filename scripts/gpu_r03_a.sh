# Round 3, first GPU call: the new C4 + R-table tests, the grid tests, then a kernel-trace profile
# of the reference grids (VG, SG) on the round-2 grid engine (the A side of the grid rework).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_rsurface.py tests/test_gpu_grid.py \
  -x -v --timeout 300 --timeout-method thread > $O/r03a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 $O/r03a_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench_configs.py --only VG,SG > $O/r03a_cfg.jsonl 2> $O/r03a_cfg.err || exit $?
cat $O/r03a_cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03a_prof -o run -- python3 bench_configs.py --only VG,SG > $O/r03a_prof.log 2>&1 || exit $?
f=$(find $O/r03a_prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -24
