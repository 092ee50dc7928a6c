set -o pipefail
mkdir -p gpurun_out/arl1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/arl1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/arl1/pytest.log; exit 1; }
tail -1 gpurun_out/arl1/pytest.log
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --config 4 --steps 30 > gpurun_out/arl1/b.json 2>gpurun_out/arl1/b.err || { echo BENCH_FAIL; tail gpurun_out/arl1/b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/arl1/b.json')); print('%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"; done
