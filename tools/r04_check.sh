#!/bin/bash
# round 4: GPU suite + smoke + config-3 bench line, then the config-5 (1 of 8)
# and config-4 (1 of 4) shard lines at 1-4 frontier chunk groups
set -o pipefail
cd "$(dirname "$0")/.."
tag=${1:-r04}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1 \
  || { tail -30 gpurun_out/$tag/tests.log; exit 1; }
tail -1 gpurun_out/$tag/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$tag/c3.json 2> gpurun_out/$tag/c3.err \
  || { tail -20 gpurun_out/$tag/c3.err; exit 1; }
python tools/bench_summary.py gpurun_out/$tag/c3.json
for nw in 1 2 3 4; do
  SGMM_FRONTIER_NW=$nw timeout -k 10 300 python -u bench.py --config 5 --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$tag/c5s8_nw$nw.json 2> gpurun_out/$tag/c5s8_nw$nw.err || { tail -20 gpurun_out/$tag/c5s8_nw$nw.err; exit 1; }
  echo "c5 1/8 nw=$nw"; python tools/bench_summary.py gpurun_out/$tag/c5s8_nw$nw.json
done
