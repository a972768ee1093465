#!/bin/bash
# Build libtrexhip variants with a compile-time diagnostic switch in tree.hip:
#   tools/build_diag.sh NAME "-DSOME_SWITCH=1"  ->  trex_amd/NAME.so
# (the TREX_MF_DIAG switches of the first LDS-staged MF, commit 25a91b1,
# produced the DESIGN.md 5.3 numbers)
set -e
cd "$(dirname "$0")/../trex_amd/csrc"
mkdir -p build/diag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -ffp-contract=off -fno-honor-nans $2 -c -o build/diag/tree_$1.o tree.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../$1.so build/sankoff.o build/sankoff_wide.o \
  build/nk.o build/plan.o build/diag/tree_$1.o
