mkdir -p gpurun_out
export TMPDIR=/tmp
ADAM_ONLY=1 timeout -k 10 200 python -u tools/time_mf_adam.py > gpurun_out/adam13.txt 2>&1 || exit 1
