# path scan: the next window gathered during the exact sum; parity, A/B vs the previous commit
set -o pipefail
mkdir -p gpurun_out/sc5
timeout -k 10 900 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sc5/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/sc5/pytest.log; exit 1; }
tail -1 gpurun_out/sc5/pytest.log
bash tools/ab_lib2.sh sc5 tools/diag/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 3 --steps 30
