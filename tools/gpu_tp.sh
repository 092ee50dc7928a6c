# config 2: table schedules (v3 default, v3i, v2) at five workgroups per CU; tail phases (register stamps)
set -o pipefail
mkdir -p gpurun_out/tp gpurun_out/sc2s
for i in 1 2; do
  for TP in v3 v3i v2; do
    SGMM_TABLE_PATH=$TP timeout -k 10 200 python -u bench.py --no-cpu-baseline --config 2 --steps 200 > gpurun_out/tp/b.json 2> gpurun_out/tp/b.err || { echo BENCH_FAIL; tail gpurun_out/tp/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/tp/b.json')); print(sys.argv[1], '%.4g'%d['value'], '%.2f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],2) for k,v in d['kernels'].items()})" $TP | tee -a gpurun_out/tp/ab.txt
  done
done
timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_t.log 2>&1 || { cat gpurun_out/sc2s/c2_t.log; exit 1; }
grep -E "tail" gpurun_out/sc2s/c2_t.log
