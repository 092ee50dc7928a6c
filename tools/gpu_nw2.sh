# frontier whole/split balance with packed slots: default vs all split vs all whole (config 3)
set -o pipefail
mkdir -p gpurun_out/nw2
for i in 1 2; do
  for NW in d 2 1; do
    if [ $NW = d ]; then unset SGMM_FRONTIER_NW; else export SGMM_FRONTIER_NW=$NW; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 3 --steps 50 > gpurun_out/nw2/b.json 2> gpurun_out/nw2/b.err || { echo BENCH_FAIL; tail gpurun_out/nw2/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/nw2/b.json')); print('NW', sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()})" $NW | tee -a gpurun_out/nw2/ab.txt
  done
done
