# quick iteration: GPU tests, microbench, bench
set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python tools/mb_rollout.py 3600 16 > gpurun_out/mb_16.json 2> gpurun_out/mb.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
