# R-stream iteration: the R-stream GPU tests, then R1 / RG / RH lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/rs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rstream.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench_configs.py --only R1,RG,RH > $O/rs.jsonl 2> $O/rs.err || exit $?
python3 -c "
import json
for l in open('$O/rs.jsonl'):
    d = json.loads(l); print(d.get('config'), {k: v for k, v in d.items() if 'per_s' in k or k in ('seconds', 'gpu_s')})"
