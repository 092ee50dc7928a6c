# Round 5: the frontier kernel with 1-16 chunk groups against the table on the
# small launches (configs 2 and 6, the config-5 1-of-8 / 1-of-16 shards).
# usage: bash tools/r05_small.sh OUTDIR
set -o pipefail
out=$1; mkdir -p "$out"
run() {  # name, env..., -- bench args
  local name=$1; shift; local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" --steps 20 --warmup 5 --no-cpu-baseline > "$out/$name.json" 2> "$out/$name.err" || { tail -5 "$out/$name.err"; return 1; }
  python tools/bench_summary.py "$out/$name.json" | sed "s/^/$name: /"
}
for c in 2 6; do
  run c${c}_table SGMM_TABLE_PATH=table -- --config $c || exit 1
  for g in 1 2 4 8 16; do run c${c}_fr$g SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=$g -- --config $c || exit 1; done
done
for s in 8 16; do
  run c5s${s}_auto SGMM_X=1 -- --config 5 --shard-of $s || exit 1
  for g in 2 4 8; do run c5s${s}_fr$g SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=$g -- --config 5 --shard-of $s || exit 1; done
done
