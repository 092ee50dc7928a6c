set -o pipefail
timeout -k 10 60 ./tools/mb/mb_fadd > gpurun_out/mb_fadd.txt 2>&1 || echo "mb_fadd failed"
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -2 gpurun_out/pytest_gpu.log
grep -q "pytest rc=0" gpurun_out/pytest_gpu.log || exit 1
timeout -k 10 300 python tools/mb_rollout.py 3600 16 1,64,1024,4096 > gpurun_out/mb_16.json 2> gpurun_out/mb.err || exit 1
timeout -k 10 300 python tools/mb_rollout.py 3600 32 64,1024 > gpurun_out/mb_32.json 2>> gpurun_out/mb.err || exit 1
