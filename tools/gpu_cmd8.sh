# round 4: GEMM version A/B (x3 v3 / v5 / v6, f32 v5 / old), NK profile, tree + nk tests
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/time_gemm_codes.py > gpurun_out/gemm8.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_nk_gpu.py tests/test_tree_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/suite8.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_nk5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_nk_eval.py > $GRAFT_REPO_ROOT/gpurun_out/prof_nk5.log 2>&1 || exit 1
