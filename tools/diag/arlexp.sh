set -o pipefail
mkdir -p gpurun_out
for v in base ONEFPT NOSTORE NOMAP; do
  if [ $v = base ]; then L=; else L=$PWD/tools/diag/libsgmm_$v.so; fi
  if [ -n "$L" ]; then export SGMM_LIB=$L; else unset SGMM_LIB; fi
  timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 5 > gpurun_out/arlexp_$v.json 2> gpurun_out/arlexp.err || { tail -20 gpurun_out/arlexp.err; exit 1; }
  python - gpurun_out/arlexp_$v.json <<'PY'
import json, sys; d=json.load(open(sys.argv[1]))
print(sys.argv[1], d["ms_per_step"], "ms", {k: round(v["avg_us"],1) for k,v in d["kernels"].items()})
PY
done
