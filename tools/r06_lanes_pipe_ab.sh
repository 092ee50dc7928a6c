# lanes scan: the chain with the next 16 values' LDS reads in flight (SGMM_LANES_PIPE) vs 32 per round trip
mkdir -p gpurun_out/lpab
one() { SGMM_LIB=tools/variants/libsgmm_$2.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $3 > gpurun_out/lpab/$1.json 2> gpurun_out/lpab/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/lpab/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items() if 'scan' in k})"; }
for i in 1 2; do
one c3_pipe_$i lpipe "--config 3" ; one c3_base_$i lbase "--config 3"
one c5s8_pipe_$i lpipe "--config 5 --shard-of 8" ; one c5s8_base_$i lbase "--config 5 --shard-of 8"
done
