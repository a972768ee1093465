# round 4: NK small-grid kernels, Gram v5 (pipelined, one wave per SIMD)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_nk_gpu.py tests/test_evals_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/nk2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/time_gemm_codes.py > gpurun_out/gemm5.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_tree_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tree5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nk2 -o run --output-format csv -- python tools/prof_nk_eval.py > gpurun_out/prof_nk2.log 2>&1 || exit 1
