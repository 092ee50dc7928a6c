set -o pipefail
mkdir -p gpurun_out/tw2
timeout -k 10 600 python -u -m pytest tests/test_gpu_ga.py -m gpu -x -q --timeout 300 --timeout-method thread -k "one_wave or modes_agree" > gpurun_out/tw2/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/tw2/pytest.log; exit 1; }
tail -1 gpurun_out/tw2/pytest.log
