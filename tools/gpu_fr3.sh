set -o pipefail
mkdir -p gpurun_out/fr3
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fr3/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E 'PASS|FAIL|Error' gpurun_out/fr3/pytest.log | tail -30; tail -40 gpurun_out/fr3/pytest.log; exit 1; }
grep -E 'frontier|paths_agree' gpurun_out/fr3/pytest.log | tail -20; tail -1 gpurun_out/fr3/pytest.log
