# Round 3: headline profiles on the current tree (pipelined + serial chunks), then C5 and C5-fused
# (kernel stats + PMC passes).  Summarise here: python scripts/summarize_prof.py r03_headline gpurun_out/r03_headline ...
set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
TAG=r03_headline bash scripts/gpu_prof_cfg.sh $B || exit $?
DCOR_SIGN_PIPELINE=0 TAG=r03_serial bash scripts/gpu_prof_cfg.sh $B || exit $?
TAG=r03_c5 bash scripts/gpu_prof_cfg.sh python3 bench_configs.py --only C5 || exit $?
TAG=r03_c5f bash scripts/gpu_prof_cfg.sh python3 bench_configs.py --only C5f || exit $?
echo all-profiled
