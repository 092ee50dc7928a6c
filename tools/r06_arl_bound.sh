# Round 6: the no-adversary frontier kernel at config 4's shapes (256 / 64 episodes of 3600 ticks,
# H = 32, ARL off: the lower bound of an adversary frontier) against the ARL table (config 4 itself).
set -o pipefail
out=gpurun_out/r06_arl; mkdir -p $out
run() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $out/$name.json 2> $out/$name.err || { tail -3 $out/$name.err; return 1; }; python tools/bench_summary.py $out/$name.json | sed "s|^$out/||"; }
run c4 --config 4 || exit 1
run c4s4 --config 4 --shard-of 4 || exit 1
run p256_table --config 6 --pop 256 --plan policy_path=table || exit 1
run p256_frontier --config 6 --pop 256 --plan policy_path=frontier || exit 1
run p64_table --config 6 --pop 64 --val-mode best --plan policy_path=table || exit 1
run p64_frontier --config 6 --pop 64 --val-mode best --plan policy_path=frontier || exit 1
for g in 2 4 8; do run p256_fr_g$g --config 6 --pop 256 --plan policy_path=frontier,groups=$g || exit 1; done
for g in 4 8 16; do run p64_fr_g$g --config 6 --pop 64 --val-mode best --plan policy_path=frontier,groups=$g || exit 1; done
