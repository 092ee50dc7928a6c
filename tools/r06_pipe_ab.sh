# Round 6: the sequential chain with the next batch's LDS reads in flight (SGMM_SEQ_PIPE) vs 32 per round trip
out=gpurun_out/r06_pipe; mkdir -p $out
run() { local name=$1 lib=$2; shift 2; SGMM_LIB=tools/variants/libsgmm_$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err || { tail -3 $out/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$out/$name.json').read().strip().split('\n')[-1]); print('$name', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items() if 'scan' in k})"; }
for i in 1 2; do for lib in base6 pipe16 pipe8; do
  run c3_${lib}_$i $lib --config 3 --plan fused_scan=0 || exit 1
  run c5s8_${lib}_$i $lib --config 5 --shard-of 8 --plan fused_scan=0 || exit 1
done; done
