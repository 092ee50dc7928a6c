# scan: trade-count rows loaded with the chunk maps; parity, A/B (P=4096 and config 3)
set -o pipefail
mkdir -p gpurun_out/sc6
timeout -k 10 900 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sc6/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/sc6/pytest.log; exit 1; }
tail -1 gpurun_out/sc6/pytest.log
bash tools/ab_lib2.sh sc6a tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 2 --pop 4096 --steps 30 || exit 1
bash tools/ab_lib2.sh sc6b tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 1 --config 3 --steps 30
