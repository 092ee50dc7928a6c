# config 2: table kernel at 5 waves per SIMD (96 VGPRs, genome staged in the reward LDS); parity + A/B + stamps
set -o pipefail
mkdir -p gpurun_out/occ5 gpurun_out/sc2s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_frontier.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/occ5/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/occ5/pytest.log; exit 1; }
tail -1 gpurun_out/occ5/pytest.log
bash tools/ab_lib2.sh occ5a tools/mb/libsgmm_base.so deep-reinforcement-learning-based-signal-gated-market-making_amd/libsgmm.so 3 --config 2 --steps 200 || exit 1
STAMP_OUT=gpurun_out/sc2s/c2_occ5.npz timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_occ5.log 2>&1 || { cat gpurun_out/sc2s/c2_occ5.log; exit 1; }
grep -E "table|waves per" gpurun_out/sc2s/c2_occ5.log
