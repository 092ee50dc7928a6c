#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 3 --steps 20 --warmup 5 > gpurun_out/f3_$lab.json 2>/dev/null || { echo "FAIL $lab"; exit 1; }
  python - $lab gpurun_out/f3_$lab.json <<'PY'
import json, sys; d=json.load(open(sys.argv[2]))
print(sys.argv[1], f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, flush=True)
PY
}
run base SGMM_FRONTIER_FUSED=0
run st50 SGMM_FRONTIER_FUSED=1 SGMM_SCAN_START=0.5
run st80 SGMM_FRONTIER_FUSED=1 SGMM_SCAN_START=0.8
run st95 SGMM_FRONTIER_FUSED=1 SGMM_SCAN_START=0.95
run st95s256 SGMM_FRONTIER_FUSED=1 SGMM_SCAN_START=0.95 SGMM_SCANNERS=256
SGMM_SCAN_START=0.8 timeout -k 10 300 python -u tools/mb_fused_timeline.py 10 2>&1 | grep -v amdgpu.ids
