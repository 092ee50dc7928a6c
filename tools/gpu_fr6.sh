set -o pipefail
mkdir -p gpurun_out/fr6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fr6/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/fr6/pytest.log; exit 1; }
tail -1 gpurun_out/fr6/pytest.log
timeout -k 10 200 python -u tools/mb_frontier_timeline.py 512 || exit 1
bash tools/ab_lib2.sh fr6 tools/mb/libsgmm_fr1.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 1 --config 3 --steps 30
