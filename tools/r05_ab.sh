# Round-5 A/B on one GPU box: alternate bench runs of variants given as
# NAME=ENV_ASSIGNMENTS (space-separated, ';' for none), ROUNDS times each.
# usage: bash tools/r05_ab.sh OUTDIR ROUNDS "bench args" "new=;" "head=SGMM_LIB=tools/variants/libsgmm_head.so" ...
set -e
out=$1; rounds=$2; args=$3; shift 3
mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}; [ "$envs" = ";" ] && envs=""
    env $envs timeout -k 10 240 python bench.py $args --no-cpu-baseline > "$out/${name}_$r.json" 2> "$out/${name}_$r.err"
    python tools/bench_summary.py "$out/${name}_$r.json" | sed "s/^/$name r$r: /"
  done
done
