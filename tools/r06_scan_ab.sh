# Round 6: path-scan workgroup width per shape (plan override scan_threads), 20 generations each
set -o pipefail
out=gpurun_out/r06_scanw; mkdir -p $out
run() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err || { tail -3 $out/$name.err; return 1; }; python tools/bench_summary.py $out/$name.json | sed "s|^$out/||" | cut -c1-200; }
for w in 64 256 512 1024; do run c5s16_w$w --config 5 --shard-of 16 --plan scan_threads=$w || exit 1; done
for w in 64 256 512; do run c5s8_w$w --config 5 --shard-of 8 --plan scan_threads=$w || exit 1; done
for w in 64 256 512 1024; do run c4s4_w$w --config 4 --shard-of 4 --plan scan_threads=$w || exit 1; done
for w in 256 512 1024; do run c2_w$w --config 2 --plan scan_threads=$w || exit 1; done
