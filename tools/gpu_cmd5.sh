# round 4: full GPU suite, default bench, rocprof of the bench, GEMM PMC A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/suite5.log 2>&1
rc=$?
timeout -k 10 400 python -u bench.py > gpurun_out/bench5.json 2> gpurun_out/bench5.err || exit 1
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench5_rocprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/bench5_rocprof.err || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 bash tools/pmc_gemm_ab.sh > gpurun_out/pmcab.log 2>&1 || exit 1
exit $rc
