#!/bin/bash
# bench lines under the library's env knobs: bash tools/r04_knobs.sh <tag> "<name>|<env>|<bench args>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
mkdir -p gpurun_out/$tag
for spec in "$@"; do
  IFS='|' read -r name envs bargs <<< "$spec"
  env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $bargs > gpurun_out/$tag/$name.json 2> gpurun_out/$tag/$name.err \
    || { tail -20 gpurun_out/$tag/$name.err; exit 1; }
  python tools/bench_summary.py gpurun_out/$tag/$name.json
done
