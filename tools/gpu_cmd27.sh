mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tree_gpu.py tests/test_nk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/suite27.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke27.log 2>&1 || exit 1
