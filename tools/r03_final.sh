#!/bin/bash
# round 3: what the driver runs at round end -- every GPU test, smoke(), the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_final_tests.log 2>&1 \
  || { tail -30 gpurun_out/r03_final_tests.log; exit 1; }
tail -1 gpurun_out/r03_final_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err \
  || { tail -20 gpurun_out/r03_final_bench.err; exit 1; }
python tools/bench_summary.py gpurun_out/r03_final_bench.json
