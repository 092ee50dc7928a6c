#!/bin/bash
# round 3: GPU tests (every -m gpu test) then the driver's bench command, each under its own limit
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/r03_tests.log 2>&1 || { tail -30 gpurun_out/r03_tests.log; exit 1; }
tail -3 gpurun_out/r03_tests.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail -20 gpurun_out/r03_bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open("gpurun_out/r03_bench.json"))
print(d["value"]/1e9, "G", d["ms_per_step"], "ms", {k: round(v["avg_us"],1) for k,v in d["kernels"].items()}, d["roofline"]["frac"])
PY
