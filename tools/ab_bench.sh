# Alternating A/B bench of two libraries on one box.  Usage: bash tools/ab_bench.sh <libA> <libB> [rounds]
set -o pipefail
A=$1; B=$2; N=${3:-3}
mkdir -p gpurun_out/ab
for i in $(seq 1 $N); do
  for L in $A $B; do
    SGMM_LIB=$L timeout -k 10 120 python -u bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo BENCH_FAIL $L; tail gpurun_out/ab/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()})" $L
  done
done
