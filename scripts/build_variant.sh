# Build an A/B variant of the engine with extra compile-time flags into dcor/libdcor_<name>.so
# (run with DCOR_LIB=<that path>): bash scripts/build_variant.sh <name> "<-D flags>"
# Only dcor_fused.hip and dcor_premat.hip take the flags; the other objects are the default
# build's (python -c "import __graft_entry__ as g; g.build()" first).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/distributed-correlation_amd/csrc
O=$R/distributed-correlation_amd/build/obj
V=$R/distributed-correlation_amd/build/var_$1
mkdir -p $V
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
/opt/rocm/bin/hipcc $F $2 -c -o $V/dcor_fused.hip.o $C/dcor_fused.hip &
/opt/rocm/bin/hipcc $F $2 -c -o $V/dcor_premat.hip.o $C/dcor_premat.hip &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/distributed-correlation_amd/dcor/libdcor_$1.so \
  $V/dcor_fused.hip.o $V/dcor_premat.hip.o $O/dcor_rstream.hip.o $O/dcor_capi.cpp.o $O/dcor_grid.cpp.o $O/dcor_mtjump.cpp.o \
  $O/dcor_stamp.cpp.o
