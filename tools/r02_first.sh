# Round-2 first GPU pass: every -m gpu test, the default (config 3) bench line
# with the CPU baseline, then a rocprofv3 kernel-trace summary of the bench.
# Usage (on the GPU box): bash tools/r02_first.sh <tag>
set -o pipefail
T=${1:-r02a}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err \
    || { echo BENCH_FAIL; tail -20 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt -o bench -- \
    python bench.py --steps 50 --warmup 5 --no-cpu-baseline --profile-steps 10 > gpurun_out/$T/kt_bench.json 2> gpurun_out/$T/kt.err \
    || { echo "kernel-trace failed"; tail gpurun_out/$T/kt.err; exit 1; }
find gpurun_out/$T/kt -name '*kernel_stats.csv' -exec cat {} \;
echo done
