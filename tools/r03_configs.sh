#!/bin/bash
# round 3: bench lines for configs 2 and 4, and one rank's shard of configs 4 / 5 (table vs frontier)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
summ() {
python - "$1" <<'PY'
import json, sys; d=json.load(open(sys.argv[1]))
r = d["roofline"]
print(sys.argv[1].split("/")[-1], round(d["value"]/1e9, 3), "G", round(d["ms_per_step"]*1e3, 1), "us/gen", {k: round(v["avg_us"],1) for k,v in d["kernels"].items()}, "frac", round(r["frac"], 4), flush=True)
PY
}
b() {  # out, env..., -- bench args
  local out=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --profile-steps 20 "$@" \
    > gpurun_out/$out.json 2> gpurun_out/$out.err || { tail -20 gpurun_out/$out.err; exit 1; }
  summ gpurun_out/$out.json
}
for c in ${CONFIGS:-2 4}; do b r03_c$c X=1 -- --config $c; done
[ -n "${ONLY_CONFIGS:-}" ] && exit 0
# the table / frontier crossover: the training launch on the frontier kernel from
# SGMM_FRONTIER_MIN_EPS episodes (the validation launches stay on the table)
for N in ${SHARDS5:-32 16 8 4}; do
  b r03_c5_shard${N}_table SGMM_FRONTIER_MIN_EPS=1000000 -- --config 5 --shard-of $N
  b r03_c5_shard${N}_frontier SGMM_FRONTIER_MIN_EPS=64 -- --config 5 --shard-of $N
done
b r03_c4_shard4 X=1 -- --config 4 --shard-of 4
