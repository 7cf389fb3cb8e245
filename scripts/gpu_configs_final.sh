# Every bench_configs line on the final round-2 tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u bench_configs.py > $O/configs_final.jsonl 2> $O/configs_final.err || exit $?
python3 -c "
import json
for l in open('$O/configs_final.jsonl'):
    d = json.loads(l); print(d.get('config'), {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if 'per_s' in k or 'frac' in k})"
