#!/bin/bash
# A/B of an environment switch on the config-3 bench, alternating on one box:
#   bash tools/r03_ab.sh VAR VAL_A VAL_B ROUNDS [bench args]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=$1; A=$2; B=$3; R=$4; shift 4
for r in $(seq 1 $R); do
  for val in $A $B; do
    env $V=$val timeout -k 10 300 python -u bench.py --no-cpu-baseline --profile-steps 3 "$@" > gpurun_out/ab_${V}_${val}_$r.json 2>/dev/null || exit 1
    python - "$V=$val" gpurun_out/ab_${V}_${val}_$r.json <<'PY'
import json, sys; d=json.load(open(sys.argv[2]))
print(sys.argv[1], f"{d['value']/1e9:.2f} G {d['ms_per_step']*1e3:.1f} us/gen", {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, flush=True)
PY
  done
done
