# final tree: GPU suite, smoke, default bench (config 3 with the CPU baseline)
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/final/pytest.log; exit 1; }
tail -1 gpurun_out/final/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo BENCH_FAIL; tail gpurun_out/final/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/bench.json')); print('c3', '%.4g'%d['value'], '%.3f ms'%d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
