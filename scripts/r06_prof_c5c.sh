# Counters of the C5-continuous kernels on the current tree (serial profile passes).
set -o pipefail
export TMPDIR=/tmp
bash scripts/prof.sh r06w_c5c trace,sq,mix,lds,tcp,fetch -- bench_configs.py --only C5c || exit $?
cat profiles/r06w_c5c_summary.md | head -14
python3 -c "
import json; d=json.load(open('profiles/r06w_c5c_summary.json'))
for k,v in d['kernels'].items():
    if 'tiled' in k or 'subg_int' in k: print(k[:60], {x: v[x] for x in v if x.startswith('SQ_') or x.startswith('pmc') or 'per' in x})
"
