# Round 3: the R-stream jump path (segment-parallel MT19937 from jump-ahead windows, pointer-
# doubling walk) and the coded-panel finite clip: parity tests, then R1 / RG / RH / C5 timed and
# kernel-traced.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_rstream.py tests/test_gpu_hrs.py -x -v --timeout 200 --timeout-method thread > $O/rsj_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 $O/rsj_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench_configs.py --only R1,RG,RH,C5,C5f > $O/rsj_cfg.jsonl 2> $O/rsj_cfg.err || exit $?
cat $O/rsj_cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rsj_prof -o run -- python3 bench_configs.py --only R1 > $O/rsj_prof.log 2>&1 || exit $?
f=$(find $O/rsj_prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -24
