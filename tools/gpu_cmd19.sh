mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_mix_small.sh C3 > gpurun_out/pmc19.log 2>&1 || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof19_c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_c5.py > $GRAFT_REPO_ROOT/gpurun_out/prof19_c5.log 2>&1 || exit 1
