#!/bin/bash
# Diagnostic build of the staged kernel with phase timestamps:
#   tools/build_diag_staged.sh  ->  trex_amd/libtrex_stagetime.so
set -e
cd "$(dirname "$0")/../trex_amd/csrc"
mkdir -p build/diag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -ffp-contract=off -fno-honor-nans -DTREX_STAGED_TIMING -c -o build/diag/staged_t.o sankoff_staged.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libtrex_stagetime.so build/sankoff.o \
  build/sankoff_wide.o build/diag/staged_t.o build/tree.o build/nk.o build/rundp.o build/plan.o \
  build/comm.o -ldl
