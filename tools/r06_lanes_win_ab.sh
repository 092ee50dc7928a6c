# lanes scan (2 episodes per workgroup on config 3): 256- vs 512-tick windows
mkdir -p gpurun_out/winab
one() { SGMM_LIB=tools/variants/libsgmm_$2.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $3 > gpurun_out/winab/$1.json 2> gpurun_out/winab/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/winab/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items() if 'scan' in k})"; }
for i in 1 2; do for v in win256 win512; do
one c3_${v}_$i $v "--config 3"
one c5s8_${v}_$i $v "--config 5 --shard-of 8"
done; done
