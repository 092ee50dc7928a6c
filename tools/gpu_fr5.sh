set -o pipefail
mkdir -p gpurun_out/fr5
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fr5/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/fr5/pytest.log; exit 1; }
tail -1 gpurun_out/fr5/pytest.log
bash tools/ab_lib2.sh fr5 tools/mb/libsgmm_fr1.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 3 --steps 30 || exit 1
timeout -k 10 200 python -u tools/mb_frontier_stamps.py 512 0.05 || exit 1
timeout -k 10 200 python -u tools/mb_frontier_stamps.py 16 0.05
