#!/bin/bash
# round 3: frontier layer 3 as packed fma (SGMM_L3_PACKED) against the default, alternating, config 3;
# then the frontier GPU tests on the packed library
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2 3; do
  for L in base l3p; do
    SGMM_LIB=tools/diag/libsgmm_$L.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 20 \
      > gpurun_out/l3_$L.json 2> gpurun_out/l3.err || { tail gpurun_out/l3.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[2])); r=d['roofline']['launch_us_over_timed_window']; print(sys.argv[1], '%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()}, round(r['first']), round(r['last']))" $L gpurun_out/l3_$L.json
  done
done
SGMM_LIB=tools/diag/libsgmm_l3p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
