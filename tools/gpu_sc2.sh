set -o pipefail
mkdir -p gpurun_out/sc2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sc2/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/sc2/pytest.log; exit 1; }
tail -1 gpurun_out/sc2/pytest.log
for C in 3 5 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $C --steps 20 > gpurun_out/sc2/b$C.json 2>gpurun_out/sc2/b$C.err || { echo BENCH_FAIL $C; tail gpurun_out/sc2/b$C.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sc2/b$C.json')); print('config $C', '%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'])"
done
