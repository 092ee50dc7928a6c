#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mb_heavy_predict.py 0 5 15 30 2>&1 | grep -v amdgpu.ids
