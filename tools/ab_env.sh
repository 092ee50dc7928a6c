# Alternating A/B bench of two environment settings on one box.
# Usage: bash tools/ab_env.sh <tag> "<envA>" "<envB>" <rounds> <bench args...>
#   e.g. bash tools/ab_env.sh ab1 "SGMM_TABLE_PATH=v2" "SGMM_TABLE_PATH=v3" 2 --config 3 --steps 50
set -o pipefail
T=$1; A=$2; B=$3; N=$4
shift 4
mkdir -p gpurun_out/$T
for i in $(seq 1 $N); do
  for E in "$A" "$B"; do
    env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err \
        || { echo "BENCH_FAIL $E"; tail gpurun_out/$T/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/$T/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'])" "$E" | tee -a gpurun_out/$T/ab.txt
  done
done
