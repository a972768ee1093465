mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1 0 1; do
  TREX_NK_PP=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-c5 --no-c2 --no-c3 --no-ragged --no-shard --no-e2e --steps 5 > gpurun_out/nk23.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/nk23.json')); print('TREX_NK_PP=$v', {k: round(v['ms_per_step'],4) for k,v in d['nk'].items() if isinstance(v, dict) and 'ms_per_step' in v})" >> gpurun_out/nk23.txt
done
TREX_NK_PP=1 timeout -k 10 300 python -u -m pytest tests/test_nk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nk23_tests.log 2>&1 || exit 1
