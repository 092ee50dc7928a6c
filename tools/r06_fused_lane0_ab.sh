# fused scan: the chain on lane 0 only (SGMM_FUSED_LANE0) vs on all 64 lanes
mkdir -p gpurun_out/fl0
one() { SGMM_LIB=tools/variants/libsgmm_$2.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $3 > gpurun_out/fl0/$1.json 2> gpurun_out/fl0/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/fl0/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step']*1000,1), {k: round(v['avg_us'],1) for k,v in d['kernels'].items() if 'frontier' in k or 'scan' in k})"; }
for i in 1 2; do for v in fl0 flall; do
one c5_${v}_$i $v "--config 5"
one c3w_${v}_$i $v "--config 3 --plan tail=0"
one c5s8_${v}_$i $v "--config 5 --shard-of 8 --plan fused_scan=1"
done; done
