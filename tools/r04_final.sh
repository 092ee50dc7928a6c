#!/bin/bash
# round 4 final evidence: GPU suite + smoke, the default bench line (config 3 with
# the CPU baseline), kernel stats + PMC + counters per config, the reference
# pipeline shape at 20 and 100 generations.  Everything under gpurun_out/r04f_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/tests.log 2>&1 \
  || { tail -30 gpurun_out/r04f/tests.log; exit 1; }
tail -1 gpurun_out/r04f/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f/smoke.log 2>&1 || { tail -5 gpurun_out/r04f/smoke.log; exit 1; }
tail -1 gpurun_out/r04f/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04f/c3_default.json 2> gpurun_out/r04f/c3_default.err || { tail -20 gpurun_out/r04f/c3_default.err; exit 1; }
python tools/bench_summary.py gpurun_out/r04f/c3_default.json
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/r04f/c3_100gen.json 2> gpurun_out/r04f/c3_100gen.err || { tail -20 gpurun_out/r04f/c3_100gen.err; exit 1; }
python tools/bench_summary.py gpurun_out/r04f/c3_100gen.json
for spec in "c3|--config 3" "c4|--config 4" "c5s8|--config 5 --shard-of 8" "c4s4|--config 4 --shard-of 4" "c2|--config 2" "c6|--config 6" "c7|--config 7"; do
  IFS='|' read -r name args <<< "$spec"
  bash tools/r04_profile.sh r04f_$name $args > gpurun_out/r04f/profile_$name.log 2>&1 || { tail -20 gpurun_out/r04f/profile_$name.log; exit 1; }
  head -1 gpurun_out/r04f/profile_$name.log
done
for c in 6 7; do
  for g in 20 100; do
    timeout -k 10 300 python -u bench.py --config $c --steps $g --warmup 5 > gpurun_out/r04f/c${c}_g$g.json 2> gpurun_out/r04f/c${c}_g$g.err \
      || { tail -20 gpurun_out/r04f/c${c}_g$g.err; exit 1; }
    python tools/bench_summary.py gpurun_out/r04f/c${c}_g$g.json
  done
done
