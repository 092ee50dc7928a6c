# relu on the float pipe: parity suite, then A/B against the integer-max build (configs 3, 2)
set -o pipefail
mkdir -p gpurun_out/relu
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/relu/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/relu/pytest.log; exit 1; }
tail -1 gpurun_out/relu/pytest.log
bash tools/ab_lib2.sh relu tools/mb/libsgmm_reluint.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 3 --steps 30 || exit 1
bash tools/ab_lib2.sh relu2 tools/mb/libsgmm_reluint.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 2 --steps 200
