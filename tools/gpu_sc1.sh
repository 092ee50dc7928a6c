set -o pipefail
mkdir -p gpurun_out/sc1
SGMM_SCAN_THREADS=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frontier.py tests/test_gpu_ga.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sc1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/sc1/pytest.log; exit 1; }
tail -1 gpurun_out/sc1/pytest.log
for i in 1 2; do for E in SGMM_SCAN_THREADS=256 SGMM_SCAN_THREADS=64; do
  env $E timeout -k 10 200 python bench.py --no-cpu-baseline --config 3 --steps 30 > gpurun_out/sc1/b.json 2>gpurun_out/sc1/b.err || { echo BENCH_FAIL; tail gpurun_out/sc1/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sc1/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" $E
done; done
