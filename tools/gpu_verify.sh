# Full verification on the GPU box: smoke, gpu tests, bench, bundle bench.
# Usage: bash tools/gpu_verify.sh <tag>
set -o pipefail
T=${1:-v}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/$T/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$T/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/$T/bench.err; exit 1; }
cat gpurun_out/$T/bench.json
timeout -k 10 300 python -u tools/bench_bundle.py > gpurun_out/$T/bundle.jsonl 2> gpurun_out/$T/bundle.err || { echo BUNDLE_FAIL; tail -30 gpurun_out/$T/bundle.err; exit 1; }
cat gpurun_out/$T/bundle.jsonl
echo VERIFY_DONE
