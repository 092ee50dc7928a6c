# the round-1 P=4096 scaling point (config-2 shape: H=16, 3600 + 720 ticks) in both validation modes
set -o pipefail
mkdir -p gpurun_out/p4096
for V in best fused; do
  timeout -k 10 300 python bench.py --config 2 --pop 4096 --steps 30 --no-cpu-baseline --val-mode $V > gpurun_out/p4096/$V.json 2> gpurun_out/p4096/$V.err || { echo FAIL; tail gpurun_out/p4096/$V.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/p4096/$V.json')); print('$V', '%.4g'%d['value'], '%.3f ms'%d['ms_per_step'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items()}, 'frac %.3f'%d['roofline']['frac'])"
done
