#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_fr_tests.log 2>&1 || { tail -40 gpurun_out/r03_fr_tests.log; exit 1; }
tail -1 gpurun_out/r03_fr_tests.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 3 --steps 20 --warmup 5 > gpurun_out/ab6_$lab.json 2>/dev/null || { echo "FAIL $lab"; exit 1; }
  python - $lab gpurun_out/ab6_$lab.json <<'PY'
import json, sys; d=json.load(open(sys.argv[2]))
print(sys.argv[1], f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, flush=True)
PY
}
for r in 1 2; do
run nw1_$r SGMM_FRONTIER_NW=1
run nw3_$r SGMM_FRONTIER_NW=3
run fused_$r SGMM_FRONTIER_FUSED=1
done
