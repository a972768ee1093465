#!/bin/bash
# A/B the C5 line across library builds on the same box.
# usage: tools/ab_c5_libs.sh lib1.so lib2.so ... (reps via REPS; extra env per run via ENVS)
cd "$(dirname "$0")/.."
ARGS=${BENCH_ARGS:---no-cpu-baseline --no-c2 --no-c3 --no-nk --no-ragged --no-shard --no-e2e --steps 5}
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    TREX_HIP_LIB=$lib timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab.json || exit 1
    python -c "
import json,sys
d=json.load(open(sys.argv[1]))
c=d['c5']
print(sys.argv[2], 'c5 %.3f ms gram %.1f mf %.1f us' % (c['ms_per_step'], c['kernels']['gram']['us'], c['kernels']['mf']['us']))" gpurun_out/ab.json "$lib"
  done
done
