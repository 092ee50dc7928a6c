# configs 2 and 6 (the reference's P = 50): the table variants
mkdir -p gpurun_out/sab
one() { timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $2 > gpurun_out/sab/$1.json 2> gpurun_out/sab/$1.err || { tail -3 gpurun_out/sab/$1.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sab/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step']*1000,1), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"; }
for i in 1 2; do
one c6_def_$i "--config 6" ; one c6_sp_$i "--config 6 --plan table_sp=1" ; one c6_fr16_$i "--config 6 --plan policy_path=frontier,groups=16,lane_split=4"
one c2_def_$i "--config 2" ; one c2_sp_$i "--config 2 --plan table_sp=1"
done
