set -o pipefail
mkdir -p gpurun_out/d1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/mb_scan_stamps.py > gpurun_out/d1/scan_stamps.txt 2>&1 || { echo SCANSTAMP_FAIL; exit 1; }
timeout -k 10 200 python -u tools/mb_table_stamps.py > gpurun_out/d1/table_stamps.txt 2>&1 || { echo TSTAMP_FAIL; exit 1; }
for P in 64 256 1024 4096; do
timeout -k 10 200 python -u bench.py --pop $P --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/d1/bench_p$P.json 2> gpurun_out/d1/bench_p$P.err || { echo BENCH_FAIL $P; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d1/bundle_kt -o bundle -- python -u tools/bench_bundle.py > gpurun_out/d1/bundle_prof.jsonl 2> gpurun_out/d1/bundle_prof.err || { echo BUNDLEPROF_FAIL; exit 1; }
echo DIAG_DONE
