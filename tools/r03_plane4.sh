#!/bin/bash
# round 3: frontier planes in 4-tick groups (default) against round 2's rows (SGMM_PLANE1), alternating, config 3
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p4_tests.log 2>&1 || { tail -30 gpurun_out/p4_tests.log; exit 1; }
tail -1 gpurun_out/p4_tests.log
for i in 1 2 3; do
  for L in p1 p4; do
    SGMM_LIB=tools/diag/libsgmm_$L.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 20 \
      > gpurun_out/p4_$L.json 2> gpurun_out/p4.err || { tail gpurun_out/p4.err; exit 1; }
    python tools/bench_summary.py gpurun_out/p4_$L.json | sed "s|gpurun_out/p4_||"
  done
done
