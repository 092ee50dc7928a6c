# the frontier path scan with 8 episodes per workgroup (chains in lanes) vs one episode per wave
mkdir -p gpurun_out/lab
one() { timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $2 > gpurun_out/lab/$1.json 2> gpurun_out/lab/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/lab/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"; }
for i in 1 2; do
one c3_lanes_$i "--config 3" ; one c3_wave_$i "--config 3 --plan lanes_scan=0"
one c5s8_lanes_$i "--config 5 --shard-of 8" ; one c5s8_wave_$i "--config 5 --shard-of 8 --plan lanes_scan=0"
one c5_lanes_$i "--config 5 --plan fused_scan=0" ; one c5_fused_$i "--config 5"
done
