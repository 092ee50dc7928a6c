# frontier walks per CU capped by unused LDS (queued walks start where a SIMD frees): config 3
set -o pipefail
mkdir -p gpurun_out/occ
for i in 1 2; do
  for PAD in 0 3200 5632; do
    SGMM_FRONTIER_LDS=$PAD timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 3 --steps 50 > gpurun_out/occ/b.json 2> gpurun_out/occ/b.err || { echo BENCH_FAIL; tail gpurun_out/occ/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/occ/b.json')); print('LDS pad', sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()})" $PAD | tee -a gpurun_out/occ/ab.txt
  done
done
