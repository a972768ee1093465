mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite25.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke25.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench25.json 2> gpurun_out/bench25.err || exit 1
