#!/bin/bash
# A/B of the coded-panel kernel variants on C5 (one GPU), with kernel stats per run.
# Usage: bash scripts/ab_c5.sh [old_tree_dir]   (old tree: a built checkout to compare against)
set -e
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
run() {  # tag, bench script, env...
  local tag=$1 script=$2; shift 2
  env "$@" timeout -k 10 120 python $script --only C5 | sed "s/^/$tag /"
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$tag -o $tag -- python $script --only C5 > /dev/null 2>&1
}
if [ -n "$1" ]; then run old $1/bench_configs.py DCOR_PREMAT_PIPELINE=0; fi
for v in 0 1 2 3; do
  run v${v} bench_configs.py DCOR_DICT_VARIANT=$v
done
