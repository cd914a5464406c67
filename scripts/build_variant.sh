#!/bin/bash
# Build an alternative librmpc for A/B timing: rmpc/librmpc_<name>.so from the current sources
# with extra compiler flags (e.g. -DRMPC_X=0).  Usage: bash scripts/build_variant.sh name [flags...]
set -e
export RMPC_DIAG=1   # the library reads its A/B knobs in diagnostics mode only
cd "$(dirname "$0")/../risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd"
name=$1; shift
make -s -j8 BUILD=build_$name HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -fno-slp-vectorize -fno-vectorize $*" LIB=rmpc/librmpc_$name.so
