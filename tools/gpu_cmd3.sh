# round 4: C3 / NK kernel profiles + the re-checked wide tests
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sankoff_wide_gpu.py -q --timeout 200 --timeout-method thread -k "c3_scale or missing" > gpurun_out/suite3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-c5 --no-c2 --no-nk --no-ragged --no-shard --no-e2e --steps 5 --warmup 2 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nk -o run --output-format csv -- python tools/prof_nk_eval.py > gpurun_out/prof_nk.log 2>&1 || exit 1
