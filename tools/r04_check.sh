#!/bin/bash
# round 4: GPU suite + smoke, then the bench lines of every config and shard shape
set -o pipefail
cd "$(dirname "$0")/.."
tag=${1:-r04}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$tag/tests.log 2>&1 \
  || { tail -30 gpurun_out/$tag/tests.log; exit 1; }
tail -1 gpurun_out/$tag/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
bench() {  # name env... (BARGS: bench arguments)
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BARGS > gpurun_out/$tag/$name.json 2> gpurun_out/$tag/$name.err \
    || { tail -20 gpurun_out/$tag/$name.err; exit 1; }
  python tools/bench_summary.py gpurun_out/$tag/$name.json
}
BARGS="" bench c3 SGMM_X=0
BARGS="--no-cpu-baseline --config 5 --shard-of 8" bench c5s8 SGMM_X=0
BARGS="--no-cpu-baseline --config 4" bench c4 SGMM_X=0
BARGS="--no-cpu-baseline --config 4 --shard-of 4" bench c4s4 SGMM_X=0
BARGS="--no-cpu-baseline --config 2" bench c2 SGMM_X=0
BARGS="--no-cpu-baseline --config 6" bench c6 SGMM_X=0
BARGS="--no-cpu-baseline --config 7" bench c7 SGMM_X=0
