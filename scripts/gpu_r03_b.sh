# Round 3: grid tests + the VG/SG lines under chunk-count variants (DCOR_GRID_MIN_CHUNKS).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_grid.py tests/test_gpu_launch_shape.py -x -q --timeout 200 --timeout-method thread > $O/r03b_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/r03b_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for mc in 1 2 4 8; do
  DCOR_GRID_MIN_CHUNKS=$mc timeout -k 10 200 python -u bench_configs.py --only VG,SG > $O/r03b_cfg_$mc.jsonl 2>> $O/r03b_cfg.err || exit $?
  echo "min_chunks=$mc"; python -c "import json,sys; [print(json.loads(l)['config'], round(json.loads(l)['reps_per_s']/1e6,2), 'M/s') for l in open('$O/r03b_cfg_$mc.jsonl')]"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03b_prof -o run -- python3 bench_configs.py --only VG > $O/r03b_prof.log 2>&1 || exit $?
f=$(find $O/r03b_prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -16
