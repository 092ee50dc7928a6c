#!/bin/bash
# round 3: frontier tick hand-offs -- every GPU test, then config 3 with hand-offs off / on, alternating
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/r03_steal_tests.log 2>&1 || { tail -40 gpurun_out/r03_steal_tests.log; exit 1; }
tail -1 gpurun_out/r03_steal_tests.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 20 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/st_$lab.json 2>/dev/null || { echo "FAIL $lab"; exit 1; }
  python - $lab gpurun_out/st_$lab.json <<'PY'
import json, sys; d=json.load(open(sys.argv[2])); r=d["roofline"]["launch_us_over_timed_window"]
print(sys.argv[1], f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, f"frontier first {r['first']:.0f} last {r['last']:.0f}", flush=True)
PY
}
for r in 1 2; do
run off_$r SGMM_FRONTIER_STEAL=0
run on_$r SGMM_FRONTIER_STEAL=1
done
