set -o pipefail
mkdir -p gpurun_out/fr1
SGMM_TABLE_PATH=frontier timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fr1/pytest_parity.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/fr1/pytest_parity.log; exit 1; }
tail -2 gpurun_out/fr1/pytest_parity.log
one() {  # one() <env> <bench args...>
  E=$1; shift
  env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/fr1/b.json 2> gpurun_out/fr1/b.err || { echo "BENCH_FAIL $E"; tail gpurun_out/fr1/b.err; return 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/fr1/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'], d['final_train_f'])" "$E"
}
for E in SGMM_TABLE_PATH=v3 SGMM_TABLE_PATH=frontier; do one $E --config 3 --steps 30 || exit 1; done
