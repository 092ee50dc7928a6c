# lanes scan on the 512-episode shard (the default there is the 4-wave scan)
mkdir -p gpurun_out/ls16
one() { timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $2 > gpurun_out/ls16/$1.json 2> gpurun_out/ls16/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/ls16/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step']*1000,1), {k: round(v['avg_us'],1) for k,v in d['kernels'].items() if 'scan' in k})"; }
for i in 1 2; do
one c5s16_lanes_$i "--config 5 --shard-of 16 --plan lanes_scan=1" ; one c5s16_def_$i "--config 5 --shard-of 16"
one c5s32_lanes_$i "--config 5 --shard-of 32 --plan lanes_scan=1" ; one c5s32_def_$i "--config 5 --shard-of 32"
done
