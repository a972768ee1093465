#!/bin/bash
# Diagnostic build of the matrix-core kernel with phase timestamps:
#   tools/build_diag_mx.sh  ->  trex_amd/libtrex_mxtime.so  (tools/mx_times.py)
set -e
cd "$(dirname "$0")/../trex_amd/csrc"
make -s
mkdir -p build/diag
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -ffp-contract=off -fno-honor-nans -DTREX_MX_TIMING -c -o build/diag/mx_t.o sankoff_mx.hip
objs=$(ls build/*.o | grep -v '/sankoff_mx.o')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libtrex_mxtime.so $objs build/diag/mx_t.o -ldl
