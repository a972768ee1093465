mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tree_gpu.py tests/test_multiproc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/suite29.log 2>&1 || exit 1
BENCH_ARGS="--no-cpu-baseline --no-c2 --no-c3 --no-nk --no-ragged --no-shard --no-e2e --steps 5" timeout -k 10 300 bash tools/ab_env.sh "TREX_SIDE_STREAM=0" "TREX_SIDE_STREAM=1" 2 > gpurun_out/ab29.txt 2>&1 || exit 1
