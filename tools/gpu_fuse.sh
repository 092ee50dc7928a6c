# frontier walk + path scan fused: parity (frontier, parity, multi, ga, rccl), A/B config 3 and P=4096
set -o pipefail
mkdir -p gpurun_out/fuse
timeout -k 10 1000 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_ga.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fuse/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/fuse/pytest.log; exit 1; }
tail -1 gpurun_out/fuse/pytest.log
bash tools/ab_env.sh fuse3 "SGMM_FRONTIER_FUSE=0" "SGMM_FRONTIER_FUSE=1" 2 --config 3 --steps 30 || exit 1
bash tools/ab_env.sh fuse4 "SGMM_FRONTIER_FUSE=0" "SGMM_FRONTIER_FUSE=1" 1 --config 2 --pop 4096 --steps 30
