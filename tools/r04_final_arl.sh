#!/bin/bash
# refresh of the adversary-path evidence after the transducer-step change
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f
for spec in "c4|--config 4" "c4s4|--config 4 --shard-of 4" "c7|--config 7"; do
  IFS='|' read -r name args <<< "$spec"
  bash tools/r04_profile.sh r04f_$name $args > gpurun_out/r04f/profile_$name.log 2>&1 || { tail -20 gpurun_out/r04f/profile_$name.log; exit 1; }
  head -1 gpurun_out/r04f/profile_$name.log
done
for g in 20 100; do
  timeout -k 10 300 python -u bench.py --config 7 --steps $g --warmup 5 > gpurun_out/r04f/c7_g$g.json 2> gpurun_out/r04f/c7_g$g.err \
    || { tail -20 gpurun_out/r04f/c7_g$g.err; exit 1; }
  python tools/bench_summary.py gpurun_out/r04f/c7_g$g.json
done
