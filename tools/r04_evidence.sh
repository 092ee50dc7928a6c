#!/bin/bash
# round 4 evidence beyond config 3: kernel stats + PMC + SQ counters for the
# ARL, shard and small configs, then the reference pipeline shape (configs 6/7)
# at 20 and 100 generations with the CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/r04_profile.sh r04_c4 --config 4 || exit 1
bash tools/r04_profile.sh r04_c4s4 --config 4 --shard-of 4 || exit 1
bash tools/r04_profile.sh r04_c5s8 --config 5 --shard-of 8 || exit 1
bash tools/r04_profile.sh r04_c2 --config 2 || exit 1
bash tools/r04_profile.sh r04_c6 --config 6 || exit 1
bash tools/r04_profile.sh r04_c7 --config 7 || exit 1
mkdir -p gpurun_out/r04_pipe
for c in 6 7; do
  for g in 20 100; do
    timeout -k 10 300 python -u bench.py --config $c --steps $g --warmup 5 > gpurun_out/r04_pipe/c${c}_g$g.json 2> gpurun_out/r04_pipe/c${c}_g$g.err \
      || { tail -20 gpurun_out/r04_pipe/c${c}_g$g.err; exit 1; }
    python tools/bench_summary.py gpurun_out/r04_pipe/c${c}_g$g.json
  done
done
