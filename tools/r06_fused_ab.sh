set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frontier.py tests/test_gpu_trained_state.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fs_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/fs_tests.log; exit 1; }
tail -3 gpurun_out/fs_tests.log
for i in 1 2; do
timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 5 > gpurun_out/fs_b_on_$i.json 2> gpurun_out/fs_b_on_$i.err || exit 1
timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 5 --plan fused_scan=0 > gpurun_out/fs_b_off_$i.json 2> gpurun_out/fs_b_off_$i.err || exit 1
done
for f in gpurun_out/fs_b_*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); print('$f', d['ms_per_step'], d['value'])"; done
