# Round-6 GPU pass: the switch-table, HRS-sharding and changed tests, then the headline and config lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_variants.py tests/test_gpu_dist.py tests/test_gpu_hrs.py tests/test_gpu_rstream.py tests/test_gpu_grid.py "tests/test_gpu_parity.py::test_bernoulli_planes_vs_regen" "tests/test_gpu_parity.py::test_fused_vs_oracle_m_over_252" "tests/test_gpu_launch_shape.py::test_headline_wide_code_window" > gpurun_out/r06/t0.log 2>&1; rc=$?; tail -3 gpurun_out/r06/t0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/bench0.log 2>&1 && tail -1 gpurun_out/r06/bench0.log | cut -c1-400 &&
timeout -k 10 400 python -u bench_configs.py --only C5,C5c,VG,C1,HS > gpurun_out/r06/cfg0.jsonl 2> gpurun_out/r06/cfg0.err && cut -c1-250 gpurun_out/r06/cfg0.jsonl
