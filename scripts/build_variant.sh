# Build an A/B variant of the engine with extra compile-time flags into dcor/libdcor_<name>.so
# (run with DCOR_LIB=<that path>): bash scripts/build_variant.sh <name> "<-D flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/distributed-correlation_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off $2 \
  -o $R/distributed-correlation_amd/dcor/libdcor_$1.so \
  $C/dcor_fused.hip $C/dcor_premat.hip $C/dcor_rstream.hip $C/dcor_capi.cpp $C/dcor_grid.cpp $C/dcor_mtjump.cpp
