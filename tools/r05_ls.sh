# Round 5: lane split (waves per 64-chunk walk) x chunk groups on config 5's shards.
set -o pipefail
out=$1; mkdir -p "$out"
run() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py --config 5 --shard-of $SH --steps 20 --warmup 5 --no-cpu-baseline > "$out/$name.json" 2> "$out/$name.err" || { tail -3 "$out/$name.err"; return 1; }; python tools/bench_summary.py "$out/$name.json" | sed "s/^/$name: /"; }
SH=8
run s8_auto SGMM_X=1 || exit 1
run s8_g1l4 SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=1 SGMM_FRONTIER_LS=4 || exit 1
run s8_g2l2 SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=2 SGMM_FRONTIER_LS=2 || exit 1
run s8_g1l2 SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=1 SGMM_FRONTIER_LS=2 || exit 1
SH=16
run s16_auto SGMM_X=1 || exit 1
run s16_g4l2 SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=4 SGMM_FRONTIER_LS=2 || exit 1
run s16_g2l4 SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=2 SGMM_FRONTIER_LS=4 || exit 1
run s16_g1l4 SGMM_TABLE_PATH=frontier SGMM_FRONTIER_NW=1 SGMM_FRONTIER_LS=4 || exit 1
