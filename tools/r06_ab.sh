# Round 6 A/B on one box: the round-5 tree (tools/variants/r5tree, built from c8f9423)
# against this tree with launch-plan overrides, alternating.
# usage: bash tools/r06_ab.sh OUTDIR ROUNDS CONFIG "name:plan" ...   (plan "" = defaults; name r5 = the old tree)
set -o pipefail
out=$1; rounds=$2; cfg=$3; shift 3; mkdir -p "$out"
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name=${spec%%:*}; plan=${spec#*:}
    if [[ "$name" == v_* ]]; then  # a variant library: tools/variants/libsgmm_<name without v_>.so
      SGMM_LIB=tools/variants/libsgmm_${name#v_}.so timeout -k 10 200 python bench.py --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline ${plan:+--plan $plan} $EXTRA > "$out/${name}_$r.json" 2> "$out/${name}_$r.err" || { tail -3 "$out/${name}_$r.err"; exit 1; }
    elif [ "$name" = r5 ]; then
      (cd tools/variants/r5tree && timeout -k 10 200 python bench.py --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline) > "$out/${name}_$r.json" 2> "$out/${name}_$r.err" || { tail -3 "$out/${name}_$r.err"; exit 1; }
    else
      timeout -k 10 200 python bench.py --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline ${plan:+--plan $plan} $EXTRA > "$out/${name}_$r.json" 2> "$out/${name}_$r.err" || { tail -3 "$out/${name}_$r.err"; exit 1; }
    fi
    python tools/bench_summary.py "$out/${name}_$r.json" | sed "s|^$out/||"
  done
done
