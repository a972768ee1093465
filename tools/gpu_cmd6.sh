# round 4: NK (fused Adam, gather-in-combine, small surrogate) + GEMM defaults, then the bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_nk_gpu.py tests/test_evals_gpu.py tests/test_tree_gpu.py tests/test_ragged_gpu.py tests/test_bigq_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/suite6.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_nk3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_nk_eval.py > $GRAFT_REPO_ROOT/gpurun_out/prof_nk3.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > gpurun_out/bench6.json 2> gpurun_out/bench6.err || exit 1
