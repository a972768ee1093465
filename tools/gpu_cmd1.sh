mkdir -p gpurun_out
for v in sitet sitetk sitetm sitetkm; do
  TREX_HIP_LIB=trex_amd/libtrex_ab_$v.so timeout -k 10 120 python -u tools/site_times.py > gpurun_out/st_$v.txt 2>&1 || exit 1
done
timeout -k 10 500 python -u tools/parity_probe.py site gemm c5 marg > gpurun_out/probe1.log 2>&1
timeout -k 10 560 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/suite1.log 2>&1
