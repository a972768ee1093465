mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=3 BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --steps 20" timeout -k 10 600 bash tools/ab_libs.sh trex_amd/libtrexhip.so trex_amd/libtrex_ab_wpe6.so trex_amd/libtrex_ab_ring2.so trex_amd/libtrex_ab_ring2w7.so > gpurun_out/ab15.txt 2>&1 || exit 1
