set -o pipefail
mkdir -p gpurun_out/rc1
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rc1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/rc1/pytest.log; exit 1; }
grep -E 'PASS|FAIL' gpurun_out/rc1/pytest.log; tail -1 gpurun_out/rc1/pytest.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rc1/pytest_all.log 2>&1 || { echo PYTEST_ALL_FAIL; tail -60 gpurun_out/rc1/pytest_all.log; exit 1; }
tail -1 gpurun_out/rc1/pytest_all.log
