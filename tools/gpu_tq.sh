# frontier kernel with 2 MFMA tiles (32 chunks) per wave: parity, A/B vs 4 tiles
set -o pipefail
mkdir -p gpurun_out/tq
timeout -k 10 900 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tq/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/tq/pytest.log; exit 1; }
tail -1 gpurun_out/tq/pytest.log
bash tools/ab_env.sh tq "SGMM_FRONTIER_TQ=4" "SGMM_FRONTIER_TQ=2" 2 --config 3 --steps 30
