# Every BASELINE config line on one GPU at its stated size -> gpurun_out/configs.jsonl
#   bash scripts/configs.sh [C1,C2,...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench_configs.py ${1:+--only $1} > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.jsonl | cut -c1-200; exit $rc
