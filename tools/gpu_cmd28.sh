mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=2 BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --no-shard --steps 20" timeout -k 10 500 bash tools/ab_libs.sh trex_amd/libtrexhip.so trex_amd/libtrex_ab_fw5.so trex_amd/libtrex_ab_fw7.so trex_amd/libtrex_ab_fw8.so > gpurun_out/ab28.txt 2>&1 || exit 1
