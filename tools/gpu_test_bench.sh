# GPU tests (optionally one file / -k filter) then the stamps + bench script.
# Usage: bash tools/gpu_test_bench.sh <tag> [pytest args...]
set -o pipefail
T=${1:-tb}; shift
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
bash tools/gpu_stamps.sh $T
