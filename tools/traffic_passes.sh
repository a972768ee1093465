#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs, kernel-trace only)
# for the bench kernels and the calibration microbenchmarks.
# usage: tools/traffic_passes.sh OUTDIR
set -e
OUT=$(realpath -m "$1")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
# calibration microbenchmarks (git-ignored binaries): build them if absent
for m in load_pattern store_pattern; do
  [ -x "$ROOT/tools/micro/$m" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -w \
    -o "$ROOT/tools/micro/$m" "$ROOT/tools/micro/$m.hip"
done
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $C -d "$OUT/pmc/$C" -o run --output-format csv -- python3 "$ROOT/tools/prof_kernels.py" --iters 5 > "$OUT/pmc_$C.log" 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/calib/load_$C" -o run --output-format csv -- "$ROOT/tools/micro/load_pattern" > "$OUT/calib_load_$C.log" 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/calib/store_$C" -o run --output-format csv -- "$ROOT/tools/micro/store_pattern" > "$OUT/calib_store_$C.log" 2>&1
done
python3 "$ROOT/tools/pmc_traffic.py" "$OUT/pmc" "$OUT/calib" --out "$OUT/traffic.json"
