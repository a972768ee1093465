mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite22.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke22.log 2>&1 || exit 1
timeout -k 10 1000 bash tools/refresh_profiles.sh gpurun_out/r04v4 > gpurun_out/refresh22.log 2>&1 || exit 1
