# GPU tests + A/B bench of kernel variants selected by env vars.
# Usage: bash tools/gpu_ab.sh <tag> "<ENV=val ...>" ["<ENV=val ...>" ...]
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
i=0
for V in "$@"; do
  i=$((i+1))
  for P in 64 4096; do
    env $V timeout -k 10 200 python -u bench.py --pop $P --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/$T/b${i}_p$P.json 2> gpurun_out/$T/b${i}_p$P.err || { echo BENCH_FAIL $V; tail -20 gpurun_out/$T/b${i}_p$P.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/$T/b${i}_p$P.json')); print('$V', $P, '%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
  done
done
echo AB_DONE
