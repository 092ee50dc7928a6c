# A/B bench of two libraries at one population size.  Usage: bash tools/ab_pop.sh <libA> <libB> <pop> [rounds]
set -o pipefail
A=$1; B=$2; P=$3; N=${4:-2}
mkdir -p gpurun_out/ab
for i in $(seq 1 $N); do
  for L in $A $B; do
    SGMM_LIB=$L timeout -k 10 150 python -u bench.py --pop $P --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { echo BENCH_FAIL $L; tail gpurun_out/ab/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/b.json')); print(sys.argv[1], sys.argv[2], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()})" $L $P
  done
done
