# ARL H=32 table at three waves per SIMD (157 VGPRs): GPU suite, config-4 A/B
set -o pipefail
mkdir -p gpurun_out/arl3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/arl3/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/arl3/pytest.log; exit 1; }
tail -1 gpurun_out/arl3/pytest.log
bash tools/ab_lib2.sh arl3a tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 4 --steps 30
