# HRS eps sweep (native segment entry): its tests, a stream-count probe, then the HS and C5 lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hrs.py tests/test_gpu_dist.py > gpurun_out/r06/hs_t.log 2>&1; rc=$?; tail -3 gpurun_out/r06/hs_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/hs_probe.py &&
timeout -k 10 300 python -u bench_configs.py --only HS,C5 > gpurun_out/r06/hs_cfg.jsonl 2> gpurun_out/r06/hs_cfg.err && cut -c1-300 gpurun_out/r06/hs_cfg.jsonl
