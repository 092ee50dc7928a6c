# packed extra slots in the frontier kernel: GPU suite, then config-3 A/B (base = unpacked)
set -o pipefail
mkdir -p gpurun_out/pk1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pk1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pk1/pytest.log; exit 1; }
tail -1 gpurun_out/pk1/pytest.log
bash tools/ab_lib2.sh pk1 tools/diag/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 3 --config 3 --steps 50
