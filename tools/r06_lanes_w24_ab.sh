# lanes scan: 2 episodes per workgroup (the rule from 2048 episodes) vs 4 on config 3, three rounds
mkdir -p gpurun_out/w24
one() { timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $2 > gpurun_out/w24/$1.json 2> gpurun_out/w24/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/w24/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items() if 'scan' in k})"; }
for i in 1 2 3; do
one c3_w2_$i "--config 3" ; one c3_w4_$i "--config 3 --plan lanes_scan=4"
done
