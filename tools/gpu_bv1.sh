# best-only validation: GPU tests of the new launches, then config 2/3/4 in both modes
set -o pipefail
mkdir -p gpurun_out/bv1
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_rccl.py tests/test_gpu_ga.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/bv1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/bv1/pytest.log; exit 1; }
tail -1 gpurun_out/bv1/pytest.log
one() {  # one() <tag> <bench args...>
  T=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bv1/$T.json 2> gpurun_out/bv1/$T.err || { echo "BENCH_FAIL $T"; tail gpurun_out/bv1/$T.err; return 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bv1/$T.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'], d['config']['val_mode'])" "$T"
}
for C in 3 2 4; do
  for V in fused best; do one c${C}_$V --config $C --steps 30 --val-mode $V || exit 1; done
done
