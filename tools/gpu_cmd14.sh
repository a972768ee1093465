mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/suite14.log 2>&1 || exit 1
TREX_HIP_LIB=trex_amd/libtrex_ab_ring7w4.so timeout -k 10 300 python -u -m pytest tests/test_sankoff_gpu.py tests/test_ragged_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/suite14r.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/time_mf_adam.py > gpurun_out/adam14.txt 2>&1 || exit 1
REPS=2 BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --steps 20" timeout -k 10 600 bash tools/ab_libs.sh trex_amd/libtrexhip.so trex_amd/libtrex_ab_fwdnt.so trex_amd/libtrex_ab_adjnt.so trex_amd/libtrex_ab_ring2.so trex_amd/libtrex_ab_ring3w4.so trex_amd/libtrex_ab_ring7w4.so > gpurun_out/ab14.txt 2>&1 || exit 1
BENCH_ARGS="--no-cpu-baseline --no-c2 --no-c3 --no-nk --no-ragged --no-shard --no-e2e --steps 5" timeout -k 10 200 bash tools/ab_env.sh "TREX_X=0" "TREX_X=1" 1 > gpurun_out/ab14c5.txt 2>&1 || exit 1
