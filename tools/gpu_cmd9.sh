mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/time_gemm_codes.py > gpurun_out/gemm9.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_tree_gpu.py -x -q --timeout 300 --timeout-method thread -k "mf or leaf_code or gram" > gpurun_out/suite9.log 2>&1 || exit 1
