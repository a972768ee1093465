mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sankoff_wide_gpu.py tests/test_sankoff_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/suite24.log 2>&1 || exit 1
for v in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-c5 --no-c2 --no-nk --no-ragged --no-shard --no-e2e --steps 5 > gpurun_out/c3_24.json || exit 1
python -c "import json; d=json.load(open('gpurun_out/c3_24.json'))['c3']; print('soft graph', round(d['soft_ms_per_step']*1e3,1), 'us; eager events', d['roofline']['launch_us'], 'us')" >> gpurun_out/c3_24.txt
done
