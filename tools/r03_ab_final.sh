#!/bin/bash
# round 3: the final tree (tools/diag/libsgmm_p4.so) against the session's starting commit 60ec987
# (tools/diag/libsgmm_s0.so), alternating, config 3 at the driver's length; then the GPU tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abf_tests.log 2>&1 || { tail -30 gpurun_out/abf_tests.log; exit 1; }
tail -1 gpurun_out/abf_tests.log
for i in 1 2 3; do
  for L in s0 p4; do
    SGMM_LIB=tools/diag/libsgmm_$L.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 20 \
      > gpurun_out/abf_$L.json 2> gpurun_out/abf.err || { tail gpurun_out/abf.err; exit 1; }
    python tools/bench_summary.py gpurun_out/abf_$L.json | sed "s|gpurun_out/abf_||"
  done
done
