# all-whole frontier default: GPU suite + smoke, then the config-3 and config-5 evidence refresh
set -o pipefail
mkdir -p gpurun_out/r02g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02g/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r02g/pytest.log; exit 1; }
tail -1 gpurun_out/r02g/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02g/smoke.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/r02g/smoke.log; exit 1; }
tail -1 gpurun_out/r02g/smoke.log
bash tools/r02_profile.sh r02g 3 || exit 1
python -c "import json; d=json.load(open('gpurun_out/r02g/c3/bench.json')); print('c3', '%.4g'%d['value'], '%.3f ms'%d['ms_per_step'], d['roofline']['frac'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r02g/c5.json 2> gpurun_out/r02g/c5.err || { echo BENCH5_FAIL; tail gpurun_out/r02g/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r02g/c5.json')); print('c5', '%.4g'%d['value'], '%.3f ms'%d['ms_per_step'], d['roofline']['frac'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
