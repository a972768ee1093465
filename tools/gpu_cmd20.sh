mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in trex_amd/libtrexhip.so trex_amd/libtrex_ab_nosplit.so trex_amd/libtrexhip.so trex_amd/libtrex_ab_nosplit.so; do
  echo "== $lib" >> gpurun_out/gemm20.txt
  TREX_HIP_LIB=$lib timeout -k 10 200 python -u tools/time_gemm_codes.py >> gpurun_out/gemm20.txt 2>&1 || exit 1
done
