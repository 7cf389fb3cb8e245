# Timing-only: pass 1's ceiling at higher occupancy (a smaller LDS ziggurat table; wrong draws).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
for l in libdcor.so libdcor_zt1k.so libdcor_zt512.so; do
  DCOR_LIB=$PWD/distributed-correlation_amd/dcor/$l timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/zt_$l.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/zt_$l.log').read().strip().splitlines()[-1]); print('$l', round(d['value']), d['roofline']['issue']['ms'])"
done
