# The engine compiled from source on the GPU box (no prebuilt objects travel: build/ is gpurun-ignored),
# then the library's hash against the shipped one, smoke, every -m gpu test and the headline bench
# on the freshly built library -> gpurun_out/r06/box_build.log.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
L=gpurun_out/r06/box_build.log
SHIPPED=$(sha256sum distributed-correlation_amd/dcor/libdcor.so | cut -d' ' -f1)
rm -f distributed-correlation_amd/dcor/libdcor.so
rm -rf distributed-correlation_amd/build
echo "shipped libdcor.so sha256 $SHIPPED (removed before the build)" > $L
date -u +"build start %FT%TZ" >> $L
timeout -k 10 900 python -u -c "import __graft_entry__ as g, time; t = time.time(); g.build_engine(force=True); print('built in %.0f s, stamp %s' % (time.time() - t, g.stamped_hash()))" >> $L 2>&1 || { tail -5 $L; exit 1; }
echo "built libdcor.so sha256 $(sha256sum distributed-correlation_amd/dcor/libdcor.so | cut -d' ' -f1)" >> $L
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 || { tail -5 $L; exit 1; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests >> $L 2>&1 || { tail -5 $L; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r06/box_build_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r06/box_build_bench.log | cut -c1-220 >> $L
grep -v "warning\|^ *[0-9]* |\|^ *|\|occupancy" $L | tail -12
