# re-entry check: GPU suite, smoke, default bench (config 3)
set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02e/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r02e/pytest.log; exit 1; }
tail -1 gpurun_out/r02e/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02e/smoke.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/r02e/smoke.log; exit 1; }
tail -1 gpurun_out/r02e/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err || { echo BENCH_FAIL; tail gpurun_out/r02e/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r02e/bench.json')); print('c3', '%.4g'%d['value'], '%.3f ms'%d['ms_per_step'], d['roofline']['frac'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
