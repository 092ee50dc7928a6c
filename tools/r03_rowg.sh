#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_rowg_tests.log 2>&1 || { tail -40 gpurun_out/r03_rowg_tests.log; exit 1; }
tail -1 gpurun_out/r03_rowg_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 3 --steps 20 --warmup 5 > gpurun_out/rowg_$r.json 2>/dev/null || exit 1
  python - gpurun_out/rowg_$r.json <<'PY'
import json, sys; d=json.load(open(sys.argv[1]))
print(f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, flush=True)
PY
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 3 --steps 20 --warmup 5 --config 5 > gpurun_out/rowg_c5.json 2>/dev/null || exit 1
python - gpurun_out/rowg_c5.json <<'PY'
import json, sys; d=json.load(open(sys.argv[1]))
print("c5", f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, flush=True)
PY
