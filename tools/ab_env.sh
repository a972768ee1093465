#!/bin/bash
# A/B the Sankoff bench under two environment settings on the same box.
# usage: tools/ab_env.sh "VAR=a" "VAR=b" [reps]
cd "$(dirname "$0")/.."
for rep in $(seq ${3:-2}); do
  for cfg in "$1" "$2"; do
    env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-c5 --no-c2 --no-c3 --steps 20 > gpurun_out/ab.json || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,1), d['roofline']['per_kernel_us'])" gpurun_out/ab.json "$cfg"
  done
done
