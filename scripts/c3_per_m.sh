# C3 per batch size: for each eps pair (m = 32, 8, 11) a serial kernel trace + SQ counters of the
# grid at 2000 replicates per cell, then the pipelined C3 line per m.
#   bash scripts/c3_per_m.sh <tag-prefix> [reps]
set -o pipefail
export TMPDIR=/tmp
P=${1:-r05_c3}; R=${2:-2000}
for e in 0.5x0.5:32 1x1:8 1.5x0.5:11; do
  eps=${e%%:*}; m=${e##*:}
  SERIAL=1 PROF_HEAD=${PROF_HEAD:-} bash scripts/prof.sh ${P}_m$m trace,sq -- bench_configs.py --only C3 --c3-reps $R --c3-eps $eps || exit $?
  timeout -k 10 300 python -u bench_configs.py --only C3 --c3-reps $R --c3-eps $eps >> gpurun_out/${P}_lines.jsonl || exit $?
done
cat gpurun_out/${P}_lines.jsonl | cut -c1-220
