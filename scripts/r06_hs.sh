# HRS eps sweep and C5-e2e on the native launch chain: their tests, the HS / C5 / C5e lines, and kernel traces of HS and C5e.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hrs.py tests/test_gpu_dist.py > gpurun_out/r06/hs_t.log 2>&1; rc=$?; tail -3 gpurun_out/r06/hs_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench_configs.py --only HS,C5,C5e > gpurun_out/r06/hs_cfg.jsonl 2> gpurun_out/r06/hs_cfg.err && cut -c1-200 gpurun_out/r06/hs_cfg.jsonl &&
bash scripts/prof.sh r06_hs trace -- bench_configs.py --only HS > /dev/null &&
bash scripts/prof.sh r06_c5e trace -- bench_configs.py --only C5e > /dev/null
