mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --no-shard --steps 20" timeout -k 10 300 bash tools/ab_env.sh "TREX_FUSED_LDS_MIN=0" "TREX_FUSED_LDS_MIN=10240" 2 > gpurun_out/ab16a.txt 2>&1 || exit 1
BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --no-shard --steps 20" timeout -k 10 300 bash tools/ab_env.sh "TREX_FUSED_LDS_MIN=8600" "TREX_FUSED_LDS_MIN=13600" 2 > gpurun_out/ab16b.txt 2>&1 || exit 1
REPS=2 BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --no-shard --steps 20" timeout -k 10 300 bash tools/ab_libs.sh trex_amd/libtrexhip.so trex_amd/libtrex_ab_ring4.so trex_amd/libtrex_ab_ring5.so > gpurun_out/ab16c.txt 2>&1 || exit 1
TREX_FUSED_LDS_MIN=10240 REPS=2 BENCH_ARGS="--no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-nk --no-ragged --no-e2e --no-shard --steps 20" timeout -k 10 300 bash tools/ab_libs.sh trex_amd/libtrex_ab_ring4.so trex_amd/libtrex_ab_ring5.so > gpurun_out/ab16d.txt 2>&1 || exit 1
