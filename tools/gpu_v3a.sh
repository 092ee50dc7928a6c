set -o pipefail
mkdir -p gpurun_out/v3a
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ga.py tests/test_gpu_multi.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/v3a/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/v3a/pytest.log; exit 1; }
tail -2 gpurun_out/v3a/pytest.log
bash tools/ab_env.sh v3a "SGMM_TABLE_PATH=v2" "SGMM_TABLE_PATH=v3" 2 --config 3 --steps 50
bash tools/ab_env.sh v3a2 "SGMM_TABLE_PATH=v2" "SGMM_TABLE_PATH=v3" 2 --config 2 --steps 400 --warmup 20
