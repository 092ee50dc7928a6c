# Round 6: path-scan episode sums, exact parallel method (seq_sum=0) against the sequential chain (1), per shape
set -o pipefail
out=gpurun_out/r06_seq; mkdir -p $out
run() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err || { tail -3 $out/$name.err; return 1; }; python tools/bench_summary.py $out/$name.json | sed "s|^$out/||" | cut -c1-230; }
for spec in "c3:--config 3" "c5:--config 5" "c5s2:--config 5 --shard-of 2" "c5s4:--config 5 --shard-of 4" "c5s8:--config 5 --shard-of 8" \
            "c5s16:--config 5 --shard-of 16" "c2:--config 2" "c6:--config 6" "c4:--config 4" "c4s4:--config 4 --shard-of 4" "c7:--config 7"; do
  name=${spec%%:*}; args=${spec#*:}
  for sq in 0 1 auto; do
    if [ $sq = auto ]; then run ${name}_auto $args || exit 1; else run ${name}_seq$sq $args --plan seq_sum=$sq || exit 1; fi
  done
done
