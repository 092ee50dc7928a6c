#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_fused_tests.log 2>&1 || { tail -40 gpurun_out/r03_fused_tests.log; exit 1; }
tail -1 gpurun_out/r03_fused_tests.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 3 --steps 20 --warmup 5 > gpurun_out/f4_$lab.json 2>/dev/null || { echo "FAIL $lab"; exit 1; }
  python - $lab gpurun_out/f4_$lab.json <<'PY'
import json, sys; d=json.load(open(sys.argv[2]))
print(sys.argv[1], f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, flush=True)
PY
}
run base SGMM_FRONTIER_FUSED=0
run f512 SGMM_FRONTIER_FUSED=1
run f256 SGMM_FRONTIER_FUSED=1 SGMM_SCANNERS=256
run f1024 SGMM_FRONTIER_FUSED=1 SGMM_SCANNERS=1024
timeout -k 10 300 python -u tools/mb_fused_timeline.py 10 2>&1 | grep -v amdgpu.ids
