set -o pipefail
mkdir -p gpurun_out/scal
for P in 64 256 1024 4096; do
  timeout -k 10 180 python -u bench.py --pop $P --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/scal/bench_pop$P.json 2> gpurun_out/scal/bench_pop$P.err || exit 1
done
for P in 64 512; do
  timeout -k 10 180 python -u bench.py --pop $P --hidden 32 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/scal/bench_h32_pop$P.json 2> gpurun_out/scal/bench_h32_pop$P.err || exit 1
done
cd gpurun_out/scal && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d prof4096 -o run -- python3 ../../bench.py --pop 4096 --steps 20 --warmup 5 --no-cpu-baseline > rp4096.json 2> rp4096.err
