#!/bin/bash
# round 3: one rank's shard of the strong-scaled configs (bench.py --shard-of N) --
# the table / frontier crossover on config 5's shards (2 assets x 4096 / N individuals)
# and config 4 at N = 4 (64 pairs)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
summ() {
python - "$1" <<'PY'
import json, sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1], round(d["value"]/1e9, 3), "G", round(d["ms_per_step"], 4), "ms", {k: round(v["avg_us"],1) for k,v in d["kernels"].items()}, round(d["roofline"]["frac"], 4))
PY
}
for N in ${SHARDS:-32 16 8 4}; do
  for tp in table frontier; do
    f=gpurun_out/r03_c5_shard${N}_$tp.json
    SGMM_TABLE_PATH=$tp timeout -k 10 300 python -u bench.py --config 5 --shard-of $N --steps 20 --warmup 5 \
      > $f 2> gpurun_out/r03_shard.err || { tail -20 gpurun_out/r03_shard.err; exit 1; }
    summ $f
  done
done
f=gpurun_out/r03_c4_shard4.json
timeout -k 10 300 python -u bench.py --config 4 --shard-of 4 --steps 20 --warmup 5 > $f 2> gpurun_out/r03_shard.err \
  || { tail -20 gpurun_out/r03_shard.err; exit 1; }
summ $f
