# tests + generation stamps + bench
set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/mb_gen_stamps.py > gpurun_out/gstamps.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
