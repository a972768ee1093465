#!/bin/bash
# One gpurun call made of named steps; every GPU step runs under its own time
# limit and the first failure ends the call (no further GPU step after it).
#
# usage (from the repo root, on the GPU box):
#   tools/gpu_run.sh TAG STEP [STEP ...]
# steps (arguments after ':' are comma-separated, commas become spaces):
#   suite[:paths]   pytest -m gpu over tests/ (or the paths) -> TAG_suite.log
#   smoke           __graft_entry__.smoke()                  -> TAG_smoke.log
#   bench[:args]    python bench.py args                     -> TAG_bench.json
#   prof[:args]     rocprofv3 --kernel-trace --stats of bench.py args
#                   -> TAG_prof/ (+ TAG_prof_by_grid.txt)
#   pmc:GROUP,WORKLOAD  tools/pmc.sh GROUP WORKLOAD -> TAG_pmc/ (+ TAG_pmc.txt summary)
#   ab:a.so,b.so | ab:A=1,A=0   tools/ab.sh over those arms -> TAG_ab.txt
# outputs land in gpurun_out/TAG_*.
set -o pipefail
TAG=$1
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=$(echo "${step#*:}" | tr ',' ' ')
  echo "[gpu_run] $TAG $name $arg"
  case "$name" in
    suite)
      timeout -k 10 900 python -u -m pytest ${arg:-tests} -m gpu --maxfail=5 -q --timeout 120 \
        --timeout-method thread > "$OUT/${TAG}_suite.log" 2>&1 || { tail -30 "$OUT/${TAG}_suite.log"; exit 1; }
      tail -3 "$OUT/${TAG}_suite.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
        > "$OUT/${TAG}_smoke.log" 2>&1 || { cat "$OUT/${TAG}_smoke.log"; exit 1; } ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > "$OUT/${TAG}_bench.json" \
        2> "$OUT/${TAG}_bench.err" || { tail -30 "$OUT/${TAG}_bench.err"; exit 1; }
      tail -c 600 "$OUT/${TAG}_bench.json" ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" $arg > "$OUT/${TAG}_prof_bench.json" \
        2> "$OUT/${TAG}_prof.err") || { tail -30 "$OUT/${TAG}_prof.err"; exit 1; }
      for csv in $(find "$OUT/${TAG}_prof" -name '*kernel_trace.csv'); do
        python3 "$ROOT/tools/kernels_by_grid.py" "$csv" >> "$OUT/${TAG}_prof_by_grid.txt" 2>&1
      done
      cat "$OUT/${TAG}_prof_by_grid.txt" ;;
    pmc)
      set -- $arg
      timeout -k 10 900 bash "$ROOT/tools/pmc.sh" "$1" "$2" "$OUT/${TAG}_pmc" > "$OUT/${TAG}_pmc.log" 2>&1 \
        || { tail -30 "$OUT/${TAG}_pmc.log"; exit 1; }
      python3 "$ROOT/tools/pmc_summary.py" "$OUT/${TAG}_pmc" > "$OUT/${TAG}_pmc.txt" 2>&1
      tail -40 "$OUT/${TAG}_pmc.txt" ;;
    ab)
      timeout -k 10 900 bash "$ROOT/tools/ab.sh" $arg > "$OUT/${TAG}_ab.txt" 2>&1 \
        || { tail -30 "$OUT/${TAG}_ab.txt"; exit 1; }
      grep -v amdgpu.ids "$OUT/${TAG}_ab.txt" | tail -20 ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
done
echo "[gpu_run] $TAG done"
