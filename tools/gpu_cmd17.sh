mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/suite17.log 2>&1 || exit 1
timeout -k 10 1000 bash tools/refresh_profiles.sh gpurun_out/r04v3 > gpurun_out/refresh17.log 2>&1 || exit 1
