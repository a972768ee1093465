mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in trex_amd/libtrexhip.so trex_amd/libtrex_ab_b128.so trex_amd/libtrex_ab_b512.so trex_amd/libtrex_ab_b1024.so trex_amd/libtrexhip.so trex_amd/libtrex_ab_b512.so; do
  echo "== $lib" >> gpurun_out/adam26.txt
  TREX_HIP_LIB=$lib timeout -k 10 120 python -u tools/time_mf_adam.py >> gpurun_out/adam26.txt 2>&1 || exit 1
done
