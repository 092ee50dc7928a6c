# full GPU suite + smoke + config 5 bench
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/full/pytest.log; exit 1; }
tail -1 gpurun_out/full/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/full/smoke.log; exit 1; }
tail -1 gpurun_out/full/smoke.log
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --steps 30 > gpurun_out/full/c5.json 2> gpurun_out/full/c5.err || { echo BENCH5_FAIL; tail gpurun_out/full/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/full/c5.json')); print('c5', '%.4g'%d['value'], '%.3f ms'%d['ms_per_step'], d['config']['val_mode'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
