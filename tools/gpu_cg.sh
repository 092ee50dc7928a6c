# compact 1D table grid (live 4-chunk groups only): parity, then A/B SGMM_TABLE_COMPACT=0/1 at config 2, stamps
set -o pipefail
mkdir -p gpurun_out/cg gpurun_out/sc2s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_frontier.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cg/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/cg/pytest.log; exit 1; }
tail -1 gpurun_out/cg/pytest.log
for i in 1 2 3; do
  for C in 0 1; do
    SGMM_TABLE_COMPACT=$C timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 2 --steps 200 > gpurun_out/cg/b.json 2> gpurun_out/cg/b.err || { echo BENCH_FAIL; tail gpurun_out/cg/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/cg/b.json')); print('COMPACT=' + sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'])" $C | tee -a gpurun_out/cg/ab.txt
  done
done
STAMP_OUT=gpurun_out/sc2s/c2_cg.npz timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_cg.log 2>&1 || { cat gpurun_out/sc2s/c2_cg.log; exit 1; }
grep -E "table|waves per" gpurun_out/sc2s/c2_cg.log
