# Serial rocprofv3 profiles (kernel trace + SQ + VALU-mix passes) of every grid / fused config line,
# the source of each line's physical fractions (bench_configs.py `physical`):
#   bash scripts/prof_configs.sh <round tag, e.g. r05> [configs, default C2,C3,C4,VG,SG,S]
# C3 and C4 run reduced (2000 replicates per n = 1e6 cell): the per-dispatch counters do not depend
# on the replicate count.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r05}; L=${2:-C2,C3,C4,VG,SG,S}
for c in ${L//,/ }; do
  lc=$(echo $c | tr 'A-Z' 'a-z')
  extra=""
  [ $c = C3 ] && extra="--c3-reps 2000"
  [ $c = C4 ] && extra="--c4-B-big 2000"
  SERIAL=1 PROF_HEAD=${PROF_HEAD:-} bash scripts/prof.sh ${T}_$lc trace,sq,mix -- bench_configs.py --only $c $extra || exit $?
done
