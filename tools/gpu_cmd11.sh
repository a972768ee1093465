mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tree_gpu.py tests/test_sankoff_gpu.py tests/test_ragged_gpu.py tests/test_configs_full_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/suite11.log 2>&1 || exit 1
BENCH_ARGS="--no-cpu-baseline --no-c2 --no-c3 --no-nk --no-ragged --no-shard --no-e2e --steps 5" timeout -k 10 400 bash tools/ab_env.sh "TREX_MF_ADAM=0" "TREX_MF_ADAM=1" 2 > gpurun_out/ab11c5.txt 2>&1 || exit 1
BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --steps 20" timeout -k 10 400 bash tools/ab_env.sh "TREX_DEFER=0" "TREX_DEFER=1" 3 > gpurun_out/ab11.txt 2>&1 || exit 1
