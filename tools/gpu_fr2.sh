set -o pipefail
mkdir -p gpurun_out/fr2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fr2/pytest_default.log 2>&1 || { echo PYTEST_FAIL default; tail -60 gpurun_out/fr2/pytest_default.log; exit 1; }
tail -1 gpurun_out/fr2/pytest_default.log
SGMM_TABLE_PATH=frontier timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fr2/pytest_frontier.log 2>&1 || { echo PYTEST_FAIL frontier; tail -60 gpurun_out/fr2/pytest_frontier.log; exit 1; }
tail -1 gpurun_out/fr2/pytest_frontier.log
