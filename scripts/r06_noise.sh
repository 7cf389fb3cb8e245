# Noise kernels (LDS log table, bit-insert sign, branch-free odd store): every -m gpu test, then HS / C5e / C5 lines and a C5e trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06/noise_t.log 2>&1; rc=$?; tail -3 gpurun_out/r06/noise_t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench_configs.py --only HS,C5e,C5 > gpurun_out/r06/noise_cfg.jsonl 2> gpurun_out/r06/noise_cfg.err && cut -c1-160 gpurun_out/r06/noise_cfg.jsonl &&
bash scripts/prof.sh r06_c5e trace,sq,mix -- bench_configs.py --only C5e > /dev/null
