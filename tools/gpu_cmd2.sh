# round-4 check: GPU suite (elementwise bars, Q <= 128, gated site launch), then the default bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/suite2.log 2>&1
rc=$?
timeout -k 10 400 python -u bench.py > gpurun_out/bench2.json 2> gpurun_out/bench2.err || exit 1
exit $rc
