# Round 3: wave-per-replicate one-pass sign kernels for small cells -- parity tests, then VG/SG
# with the pass 2 + epilogue fused (DCOR_SIGN_P2E=1) or not, then a kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grid.py tests/test_gpu_launch_shape.py \
  tests/test_gpu_c4.py tests/test_gpu_fuzz.py tests/test_gpu_more.py tests/test_gpu_rsurface.py -x -q --timeout 300 --timeout-method thread > $O/r03c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/r03c_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for f in 0 1; do
  DCOR_SIGN_P2E=$f timeout -k 10 200 python -u bench_configs.py --only VG,SG,C1,S > $O/r03c_cfg_$f.jsonl 2>> $O/r03c_cfg.err || exit $?
  echo "p2e=$f"; python -c "import json; [print(d['config'], round(d.get('reps_per_s', d.get('gpu_reps_per_s', 0))/1e6,2), 'M/s') for d in map(json.loads, open('$O/r03c_cfg_$f.jsonl'))]"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03c_prof -o run -- python3 bench_configs.py --only VG > $O/r03c_prof.log 2>&1 || exit $?
python - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r03c_prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:70].ljust(70), r['Calls'].rjust(5), f"{float(r['AverageNs'])/1e3:9.1f} us")
PY
