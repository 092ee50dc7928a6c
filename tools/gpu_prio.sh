# frontier extra slots with s_setprio 1 around the MFMA stream: GPU frontier tests, config-3 A/B
set -o pipefail
mkdir -p gpurun_out/prio
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontier.py -x -q --timeout 300 --timeout-method thread > gpurun_out/prio/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/prio/pytest.log; exit 1; }
tail -1 gpurun_out/prio/pytest.log
bash tools/ab_lib2.sh prio tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 3 --config 3 --steps 50
