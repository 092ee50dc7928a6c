#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1 || { tail -40 gpurun_out/r03_tests.log; exit 1; }
tail -1 gpurun_out/r03_tests.log
TAG=nw1 SGMM_FRONTIER_NW=1 timeout -k 10 300 python -u tools/mb_heavy_predict.py 5 15 2>&1 | grep -v amdgpu.ids
TAG=nw3 SGMM_FRONTIER_NW=3 timeout -k 10 300 python -u tools/mb_heavy_predict.py 5 15 2>&1 | grep -v amdgpu.ids
