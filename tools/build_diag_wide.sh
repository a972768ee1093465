#!/bin/bash
# Build libtrexhip variants with a compile-time switch in sankoff_wide.hip:
#   tools/build_diag_wide.sh NAME "-DTREX_DIAG_..."  ->  trex_amd/NAME.so
set -e
cd "$(dirname "$0")/../trex_amd/csrc"
mkdir -p build/diag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -ffp-contract=off -fno-honor-nans $2 -c -o build/diag/wide_$1.o sankoff_wide.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../$1.so build/sankoff.o build/diag/wide_$1.o \
  build/sankoff_staged.o build/tree.o build/nk.o build/rundp.o build/plan.o build/comm.o -ldl
