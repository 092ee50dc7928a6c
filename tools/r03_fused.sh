#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_multi.py tests/test_gpu_rccl.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_fused_tests.log 2>&1 || { tail -40 gpurun_out/r03_fused_tests.log; exit 1; }
tail -2 gpurun_out/r03_fused_tests.log
bash tools/r03_ab.sh SGMM_FRONTIER_FUSED 0 1 2 --steps 20 --warmup 5
