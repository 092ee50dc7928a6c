# bench lines for configs 3, 2, 4 with the committed PMC summaries
set -o pipefail
mkdir -p gpurun_out/bench3
for C in 3 2 4; do
  timeout -k 10 300 python bench.py --config $C > gpurun_out/bench3/c$C.json 2> gpurun_out/bench3/c$C.err || { echo "bench $C failed"; tail gpurun_out/bench3/c$C.err; exit 1; }
done
echo ok
