#!/bin/bash
# A/B the bench under two environment settings on the same box.
# usage: tools/ab_env.sh "VAR=a" "VAR=b" [reps]   (BENCH_ARGS overrides the bench flags)
cd "$(dirname "$0")/.."
ARGS=${BENCH_ARGS:---no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --steps 20}
for rep in $(seq ${3:-2}); do
  for cfg in "$1" "$2"; do
    env $cfg timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab.json || exit 1
    python -c "
import json,sys
d=json.load(open(sys.argv[1]))
extra = ''
if 'c3' in d: extra += ' c3 soft %.1f us hard %.1f us' % (d['c3']['soft_ms_per_step']*1e3, d['c3']['hard_recon_ms_per_step']*1e3)
if 'c5' in d: extra += ' c5 %.3f ms' % d['c5']['ms_per_step']
if 'c5' in d and 'kernels' in d['c5']: extra += ' (gram %.1f mf %.1f us)' % (d['c5']['kernels']['gram']['us'], d['c5']['kernels']['mf']['us'])
if 'nk' in d: extra += ' nk_dna %.3f ms' % d['nk']['dna_256x2000_q4_k4']['ms_per_step']
if 'c5_f32' in d: extra += ' c5_f32 %.3f ms' % d['c5_f32']['ms_per_step']
if 'c4_shard' in d: extra += ' shard %.1f us' % d['c4_shard']['fused_kernel_us']
print(sys.argv[2], round(d['value']/1e9,1), d['roofline']['per_kernel_us'], extra)" gpurun_out/ab.json "$cfg"
  done
done
