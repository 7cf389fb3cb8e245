# Headline: pass 2's m = 8 records through an LDS-DMA ring (DCOR_P2_RING 2-4) vs the register double
# buffer; the bit-exact headline tests under the ring first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python -u -c "
import sys; sys.path[:0] = ['.', 'distributed-correlation_amd', 'tests']
import numpy as np, dcor
from dcor import _lib
from dcor.sim import headline_cell, simulate
c = headline_cell(); ref = simulate(c, 4096, 123).cpu().numpy()
for r in ('2', '3', '4'):
    with _lib.variants(DCOR_P2_RING=r):
        got = simulate(c, 4096, 123).cpu().numpy()
    assert np.array_equal(got.view(np.int64), ref.view(np.int64)), r
print('ring bits == register path')
" || exit $?
for i in 1 2; do
for r in 0 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --variant DCOR_P2_RING=$r > $O/ring_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/ring_$r.log').read().strip().splitlines()[-1]); print('ring $r', round(d['value']), d['roofline']['issue']['ms']['pass2'])"
done
done
