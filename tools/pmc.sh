#!/bin/bash
# rocprofv3 PMC passes, one counter group per run (kernel-trace only; the
# gfx950 per-block limits of MI355X_MICROARCH.md: <= 8 SQ, 4 TCC, 2 GRBM).
#   tools/pmc.sh GROUP WORKLOAD [OUTDIR]        (on the GPU box)
# GROUP     mix   : VALU mix / SALU / LDS / VMEM / issue / wait / MFMA busy (4 passes)
#           gemm  : MFMA busy, issue, LDS conflicts (2 passes + GRBM)
#           traffic: FETCH_SIZE / WRITE_SIZE of the workload and of the calibration
#                    micro-benchmarks -> OUTDIR/traffic.json (tools/pmc_traffic.py)
# WORKLOAD  a tools/prof.py workload (c4-fused, c4-fwd, c4-bwd, c2, c3, c5, gemm, nk,
#           nk-eval; PROF_ARGS adds its flags) or "bench" (bench.py $BENCH_ARGS)
# then:     python3 tools/pmc_summary.py OUTDIR  (mean per kernel over dispatches)
set -e
G=$1; W=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(realpath -m "${3:-$ROOT/gpurun_out/pmc_${G}_$W}")
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
if [ "$W" = bench ]; then
  CMD="python3 $ROOT/bench.py ${BENCH_ARGS:---no-cpu-baseline --no-c2 --no-c3 --no-nk --no-ragged --no-shard --no-e2e --steps 2 --warmup 1 --no-settle}"
else
  CMD="python3 $ROOT/tools/prof.py $W --iters ${ITERS:-3} ${PROF_ARGS:-}"
fi
pass() {  # pass NAME "COUNTERS" [command]
  local c=${3:-$CMD}
  mkdir -p "$(dirname "$OUT/$1")"
  timeout -s KILL ${PASS_TIMEOUT:-150} rocprofv3 --kernel-trace --pmc $2 -d "$OUT/$1" -o run \
    --output-format csv -- $c > "$OUT/$1.log" 2>&1
}
case "$G" in
  mix)
    pass pass1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT"
    pass pass2 "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
    pass pass3 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
    pass pass4 "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  gemm)
    pass pass1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
    pass pass2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
    pass pass3 "GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  traffic)
    for m in load_pattern store_pattern; do  # calibration micro-benchmarks (git-ignored binaries)
      [ -x "$ROOT/tools/micro/$m" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w \
        -o "$ROOT/tools/micro/$m" "$ROOT/tools/micro/$m.hip"
    done
    for C in FETCH_SIZE WRITE_SIZE; do
      PASS_TIMEOUT=240 pass "pmc/$C" $C
      PASS_TIMEOUT=120 pass "calib/load_$C" $C "$ROOT/tools/micro/load_pattern"
      PASS_TIMEOUT=120 pass "calib/store_$C" $C "$ROOT/tools/micro/store_pattern"
    done
    python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc" "$OUT/calib" --out "$OUT/traffic.json" ;;
  *) echo "unknown group $G (mix | gemm | traffic)"; exit 2 ;;
esac
echo "pmc $G $W -> $OUT"
