# H=16 table at five workgroups per CU: full GPU suite, config-2 A/B against the previous library
set -o pipefail
mkdir -p gpurun_out/t16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t16/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/t16/pytest.log; exit 1; }
tail -1 gpurun_out/t16/pytest.log
bash tools/ab_lib2.sh t16a tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 2 --steps 200 || exit 1
bash tools/ab_lib2.sh t16b tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 1 --config 4 --steps 30
