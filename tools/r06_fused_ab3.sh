# fused vs separate path scan on config 5 whole and its 8-GPU shard
mkdir -p gpurun_out/fab
one() { timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $2 > gpurun_out/fab/$1.json 2> gpurun_out/fab/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/fab/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"; }
for i in 1 2; do
one c5_on_$i "--config 5" ; one c5_off_$i "--config 5 --plan fused_scan=0"
one c5s8_on_$i "--config 5 --shard-of 8" ; one c5s8_off_$i "--config 5 --shard-of 8 --plan fused_scan=0"
done
