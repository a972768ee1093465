#!/bin/bash
# Same-box A/B of bench lines across library builds and / or environment
# settings, REPS rounds (default 2) of one bench run per arm:
#   tools/ab.sh trex_amd/libtrexhip.so trex_amd/libtrex_ab_x.so   (TREX_HIP_LIB per arm)
#   tools/ab.sh "TREX_GRAM=3" "TREX_GRAM=5"                        (an env assignment per arm)
# BENCH_ARGS overrides the bench flags (default: the C4 line only).  One line
# per run: the arm, C4 value (1e9 updates/s), per-kernel us and whichever of
# the C3 / C5 / NK / shard lines the flags kept.
cd "$(dirname "$0")/.."
ARGS=${BENCH_ARGS:---no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --steps 20}
for rep in $(seq ${REPS:-2}); do
  for arm in "$@"; do
    if [[ "$arm" == *=* ]]; then
      env $arm timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab.json || exit 1
    else
      TREX_HIP_LIB=$arm timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab.json || exit 1
    fi
    python -c "
import json,sys
d=json.load(open(sys.argv[1]))
x = ''
if 'c4_shard' in d: x += ' shard %.1f us (step %.1f us)' % (d['c4_shard']['fused_kernel_us'], d['c4_shard']['ms_per_step'] * 1e3)
if 'c2' in d: x += ' c2 %.1f us' % (d['c2']['ms_per_step']*1e3)
if 'c3' in d: x += ' c3 soft %.1f hard %.1f us' % (d['c3']['soft_ms_per_step']*1e3, d['c3']['hard_recon_ms_per_step']*1e3)
if 'c5' in d:
    x += ' c5 %.3f ms' % d['c5']['ms_per_step']
    if 'kernels' in d['c5']: x += ' (gram %.1f mf %.1f us)' % (d['c5']['kernels']['gram']['us'], d['c5']['kernels']['mf']['us'])
if 'c5_f32' in d: x += ' c5_f32 %.3f ms' % d['c5_f32']['ms_per_step']
if 'nk' in d: x += ' nk_dna %.3f ms' % d['nk']['dna_256x2000_q4_k4']['ms_per_step']
print(sys.argv[2], round(d['value']/1e9,1), d['roofline']['per_kernel_us'], x)" gpurun_out/ab.json "$arm"
  done
done
