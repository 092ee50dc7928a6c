# one-wave tell: parity (multi / ga / rccl), A/B config 3 and P=4096
set -o pipefail
mkdir -p gpurun_out/tw
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_ga.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tw/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/tw/pytest.log; exit 1; }
tail -1 gpurun_out/tw/pytest.log
true
bash tools/ab_lib2.sh tw4 tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 2 --config 2 --pop 4096 --steps 30
