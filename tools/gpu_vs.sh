# validation scan workgroup (5 episodes of 912 ticks): 1024 threads vs 256 vs one wave (config 3)
set -o pipefail
mkdir -p gpurun_out/vs
for i in 1 2; do
  for T in 1024 256 64; do
    SGMM_SHORT_SCAN_THREADS=$T timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 3 --steps 50 > gpurun_out/vs/b.json 2> gpurun_out/vs/b.err || { echo BENCH_FAIL; tail gpurun_out/vs/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/vs/b.json')); print('val scan threads', sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()}, d['final_train_f'][:2])" $T | tee -a gpurun_out/vs/ab.txt
  done
done
