# C5-continuous: NI noise of the first ENQ batch pairs loaded before the last tile's gathers, and the
# one-round form (ONER) that frees the NI sums' registers during the sweeps: variants 2 (ENQ 3),
# 3 (ENQ 3 + ONER), 4 (ENQ 4 + ONER), 5 (ENQ 5 + ONER) against the default (1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
run() {  # name, switches...
  local n=$1; shift
  local args=()
  for v in "$@"; do args+=(--variant "$v"); done
  timeout -k 10 200 python -u bench_configs.py --only C5c "${args[@]}" > $O/c5c_$n.jsonl 2> $O/c5c_$n.err || return $?
  python3 -c "import json; d=json.loads(open('$O/c5c_$n.jsonl').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['reps_per_s'], round(d['hbm_frac'], 3))"
}
for i in 1 2; do
  run base || exit $?
  for v in 2 3 4 5; do run v$v DCOR_TILED_VARIANT=$v || exit $?; done
done
