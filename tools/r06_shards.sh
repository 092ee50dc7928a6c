# Round 6: one rank's shard of the strong-scaled configs 4 and 5 at every N (bench.py --shard-of N)
set -o pipefail
out=gpurun_out/r06_shards; mkdir -p $out
run() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err || { tail -3 $out/$name.err; return 1; }; python tools/bench_summary.py $out/$name.json | sed "s|^$out/||" | cut -c1-220; }
run c5 --config 5 || exit 1
for n in 2 4 8 16; do run c5s$n --config 5 --shard-of $n || exit 1; done
run c4 --config 4 || exit 1
for n in 2 4 8; do run c4s$n --config 4 --shard-of $n || exit 1; done
