#!/bin/bash
# One GPU call that regenerates the round's measurement artefacts:
#   rocprofv3 --kernel-trace --stats of the C4 bench and of the full bench,
#   calibrated FETCH_SIZE / WRITE_SIZE passes -> profiles/traffic.json,
#   then the full bench (which reads traffic.json) -> OUT/bench.json.
# usage: tools/refresh_profiles.sh OUTDIR      (run on the GPU box)
set -e
OUT=$(realpath -m "$1")
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
C4="--no-c2 --no-c3 --no-c5 --no-nk --no-ragged --no-cpu-baseline --steps 20"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" $C4 > "$OUT/c4_bench_under_rocprof.json" 2> "$OUT/c4.err"
bash "$ROOT/tools/pmc.sh" traffic c4 "$OUT/traffic"
cp "$OUT/traffic/traffic.json" "$ROOT/profiles/traffic.json"
timeout -k 10 400 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/all" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/all_bench_under_rocprof.json" 2> "$OUT/all.err"
echo refreshed
