#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/mb_fused_timeline.py 10 2>&1 | grep -v amdgpu.ids
