# round 4: NK per-pair kernels + small surrogate with A in LDS
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nk_gpu.py tests/test_evals_gpu.py tests/test_tree_gpu.py -x -q --timeout 300 --timeout-method thread -k "nk or landscape or parental or surrogate or evals or optimiz" > gpurun_out/suite7.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_nk4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_nk_eval.py > $GRAFT_REPO_ROOT/gpurun_out/prof_nk4.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-ragged --no-shard --no-e2e --steps 3 --warmup 1 > gpurun_out/bench7.json 2> gpurun_out/bench7.err || exit 1
