# fused vs separate path scan, config 3: plans with and without split walks
mkdir -p gpurun_out/fab
one() { timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline $2 > gpurun_out/fab/$1.json 2> gpurun_out/fab/$1.err || exit 1;
  python -c "import json; d=json.loads(open('gpurun_out/fab/$1.json').read().strip().split('\n')[-1]); print('$1', round(d['ms_per_step'],4), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})"; }
for i in 1 2; do
one on_$i "" ; one off_$i "--plan fused_scan=0"
one on_whole_$i "--plan tail=0" ; one off_whole_$i "--plan tail=0,fused_scan=0"
done
