mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in trex_amd/libtrexhip.so trex_amd/libtrex_ab_per2.so trex_amd/libtrex_ab_epi.so; do
  echo "== $lib" >> gpurun_out/mfadam12.txt
  TREX_HIP_LIB=$lib timeout -k 10 200 python -u tools/time_mf_adam.py >> gpurun_out/mfadam12.txt 2>&1 || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof12 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/time_mf_adam.py > $GRAFT_REPO_ROOT/gpurun_out/prof12.log 2>&1 || exit 1
