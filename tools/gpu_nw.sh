# frontier kernel with 1 or 2 waves per episode: parity, then A/B on config 3
set -o pipefail
mkdir -p gpurun_out/nw
timeout -k 10 900 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/nw/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/nw/pytest.log; exit 1; }
tail -1 gpurun_out/nw/pytest.log
bash tools/ab_env.sh nw "SGMM_FRONTIER_NW=1" "SGMM_FRONTIER_NW=2" 2 --config 3 --steps 30
