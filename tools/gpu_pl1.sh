set -o pipefail
mkdir -p gpurun_out/pl1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pl1/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pl1/pytest.log; exit 1; }
tail -1 gpurun_out/pl1/pytest.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/pl1; B="bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --profile-steps 5"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o p -- python $B > $D/fetch.log 2>&1 || { echo "fetch pass failed"; tail $D/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o p -- python $B > $D/write.log 2>&1 || { echo "write pass failed"; tail $D/write.log; exit 1; }
python tools/pmc_traffic.py $D/fetch $D/write $D/pmc_traffic.json | grep -A3 frontier
for i in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --config 3 --steps 30 > $D/b.json 2>$D/b.err || { echo BENCH_FAIL; tail $D/b.err; exit 1; }
python -c "import json; d=json.load(open('$D/b.json')); print('%.4g'%d['value'], '%.1f us/gen'%(d['ms_per_step']*1e3), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"; done
