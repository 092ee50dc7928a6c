# Round 6: per-generation times of the BASELINE shapes and the strong-scaled
# per-rank shards on one box (20 timed generations each, no CPU baseline).
# usage: bash tools/r06_shapes.sh OUTDIR [names...]   (default: all)
set -o pipefail
out=$1; shift; mkdir -p "$out"
want=" $* "
run() {  # name -- bench args
  local name=$1; shift; shift
  if [ "$want" != "  " ] && [[ "$want" != *" $name "* ]]; then return 0; fi
  timeout -k 10 240 python bench.py "$@" --steps 20 --warmup 5 --no-cpu-baseline > "$out/$name.json" 2> "$out/$name.err" || { tail -5 "$out/$name.err"; return 1; }
  python tools/bench_summary.py "$out/$name.json" | sed "s/^/$name: /"
}
run c3 -- --config 3 || exit 1
run c2 -- --config 2 || exit 1
run c6 -- --config 6 || exit 1
run c4 -- --config 4 || exit 1
run c4s4 -- --config 4 --shard-of 4 || exit 1
run c5 -- --config 5 || exit 1
run c5s2 -- --config 5 --shard-of 2 || exit 1
run c5s4 -- --config 5 --shard-of 4 || exit 1
run c5s8 -- --config 5 --shard-of 8 || exit 1
run c5s16 -- --config 5 --shard-of 16 || exit 1
