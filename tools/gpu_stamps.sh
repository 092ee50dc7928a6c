# Scan phase stamps (stamped build) + a short bench.  Usage: bash tools/gpu_stamps.sh <tag>
set -o pipefail
T=${1:-st}
mkdir -p gpurun_out/$T
timeout -k 10 120 python -u tools/mb_scan_stamps.py > gpurun_out/$T/scan_stamps.txt 2>&1 || { echo STAMPS_FAIL; tail gpurun_out/$T/scan_stamps.txt; exit 1; }
timeout -k 10 120 python -u tools/mb_osum2.py > gpurun_out/$T/osum.txt 2>&1 || { echo OSUM_FAIL; tail gpurun_out/$T/osum.txt; exit 1; }
SGMM_LIB=tools/mb/libsgmm_stamps.so timeout -k 10 120 python -u tools/mb_osum2.py >> gpurun_out/$T/osum.txt 2>&1 || { echo OSUM_FAIL; tail gpurun_out/$T/osum.txt; exit 1; }
timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/$T/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$T/bench.json')); print('%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
cat gpurun_out/$T/scan_stamps.txt gpurun_out/$T/osum.txt
timeout -k 10 120 python -u tools/mb_gen_stamps.py > gpurun_out/$1/gen_stamps.txt 2>&1 || { echo GEN_FAIL; tail gpurun_out/$1/gen_stamps.txt; exit 1; }; tail -8 gpurun_out/$1/gen_stamps.txt
