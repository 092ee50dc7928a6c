set -o pipefail
mkdir -p gpurun_out/v3b
one() {  # one() <env> <bench args...>
  E=$1; shift
  env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/v3b/b.json 2> gpurun_out/v3b/b.err || { echo "BENCH_FAIL $E"; tail gpurun_out/v3b/b.err; return 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/v3b/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'])" "$E"
}
for i in 1 2; do for E in SGMM_TABLE_PATH=v2 SGMM_TABLE_PATH=v3i SGMM_TABLE_PATH=v3; do
  one $E --config 3 --steps 50 || exit 1
done; done
for E in SGMM_TABLE_PATH=v2 SGMM_TABLE_PATH=v3i SGMM_TABLE_PATH=v3; do
  one $E --config 2 --steps 400 --warmup 20 || exit 1
done
