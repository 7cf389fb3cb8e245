# HRS launch chain (native, two streams): its tests, then the HS / C5 / C5e lines against the one-stream chain.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hrs.py tests/test_gpu_dist.py tests/test_gpu_variants.py > gpurun_out/r06/hs_t.log 2>&1; rc=$?; tail -3 gpurun_out/r06/hs_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench_configs.py --only HS,C5e > gpurun_out/r06/hs_cfg.jsonl 2> gpurun_out/r06/hs_cfg.err && cut -c1-200 gpurun_out/r06/hs_cfg.jsonl &&
timeout -k 10 300 python -u bench_configs.py --only HS,C5e --variant DCOR_HRS_PIPE=0 > gpurun_out/r06/hs_cfg0.jsonl 2> gpurun_out/r06/hs_cfg0.err && cut -c1-200 gpurun_out/r06/hs_cfg0.jsonl
