#!/bin/bash
# round 3: adversary path -- its GPU parity tests, then config 4 with the v3 ARL table
# against round 1's k_policy_table_mfma (SGMM_TABLE_PATH=v2), alternating
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${ARL_TESTS:-adversar or arl or config4 or length_cap or ARL}" > gpurun_out/r03_arl_tests.log 2>&1 \
  || { tail -30 gpurun_out/r03_arl_tests.log; exit 1; }
tail -3 gpurun_out/r03_arl_tests.log
for i in 1 2; do
  for tp in "" v2; do
    SGMM_TABLE_PATH=$tp timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 5 ${BENCH_ARGS:-} \
      > gpurun_out/r03_arl_${tp:-v3}_$i.json 2> gpurun_out/r03_arl.err || { tail -20 gpurun_out/r03_arl.err; exit 1; }
    python - "gpurun_out/r03_arl_${tp:-v3}_$i.json" <<'PY'
import json, sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1], d["value"]/1e9, "G", d["ms_per_step"], "ms", {k: round(v["avg_us"],1) for k,v in d["kernels"].items()}, d["roofline"]["frac"])
PY
  done
done
