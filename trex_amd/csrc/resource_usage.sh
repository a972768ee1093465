#!/bin/bash
# Print per-kernel VGPR/SGPR/scratch/occupancy of libtrexhip's device code.
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-honor-nans $RU_FLAGS -c --cuda-device-only \
  -Rpass-analysis=kernel-resource-usage "${1:-sankoff.hip}" -o /tmp/_ru.o 2>&1 |
  grep -E 'Function Name|VGPRs:|TotalSGPRs|ScratchSize|Occupancy|Spill' |
  sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//; s/^[^ ]* //; s/remark: //' |
  awk -F': ' '/Function Name/ {if (line) print line; line=$2; next} {line=line " | " $1 "=" $2} END {print line}' |
  c++filt | sed 's/trex::(anonymous namespace):://; s/(HIP_vector_type[^|]*//'
