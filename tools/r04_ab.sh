#!/bin/bash
# round 4 A/B: alternating runs of the default library and a variant (SGMM_LIB) on one config
# usage: tools/r04_ab.sh TAG VARIANT "bench args" ROUNDS
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1; var=$2; args=$3; rounds=${4:-2}
mkdir -p gpurun_out/$tag
for r in $(seq 1 $rounds); do
  for v in default $var; do
    lib=""; [ "$v" != default ] && lib="SGMM_LIB=tools/variants/libsgmm_$v.so"
    env $lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $args > gpurun_out/$tag/${v}_$r.json 2> gpurun_out/$tag/${v}_$r.err \
      || { tail -20 gpurun_out/$tag/${v}_$r.err; exit 1; }
    python tools/bench_summary.py gpurun_out/$tag/${v}_$r.json
  done
done
