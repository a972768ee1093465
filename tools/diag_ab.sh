#!/bin/bash
# A/B several builds of libtrexhip (TREX_HIP_LIB) on the C4 bench: per-kernel
# HIP-event times.  usage: tools/diag_ab.sh lib1 lib2 ... (names under trex_amd/)
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for L in "$@"; do
    TREX_HIP_LIB=trex_amd/$L.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-c5 \
      --no-c3 --no-c2 --no-nk --no-ragged --steps 20 > gpurun_out/ab.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1], d['roofline']['per_kernel_us'])" $L
  done
done
