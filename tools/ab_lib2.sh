# Alternating A/B bench of two libraries (SGMM_LIB) on one box.
# Usage: bash tools/ab_lib2.sh <tag> <libA> <libB> <rounds> <bench args...>
set -o pipefail
T=$1; A=$2; B=$3; N=$4
shift 4
mkdir -p gpurun_out/$T
for i in $(seq 1 $N); do
  for LB in $A $B; do
    SGMM_LIB=$LB timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err \
        || { echo "BENCH_FAIL $LB"; tail gpurun_out/$T/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/$T/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'])" "$LB" | tee -a gpurun_out/$T/ab.txt
  done
done
