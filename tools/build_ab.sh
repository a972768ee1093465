#!/bin/bash
# A/B builds of libtrexhip with one translation unit recompiled under extra
# defines:  tools/build_ab.sh <name> <source.hip> [-DFOO=1 ...]
#   -> trex_amd/libtrex_ab_<name>.so  (select with TREX_HIP_LIB=...)
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../trex_amd/csrc"
make -s
mkdir -p build/ab
obj=build/ab/${name}_$(basename "$src" .hip).o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -ffp-contract=off -fno-honor-nans "$@" -c -o "$obj" "$src"
objs=$(ls build/*.o | grep -v "/$(basename "$src" .hip).o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../libtrex_ab_${name}.so $objs "$obj" -ldl
