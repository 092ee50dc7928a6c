# Round 6: frontier spill parity tests, then config 3 with spill deadlines (us) against the round-5 tree.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_frontier.py -x -q --timeout 120 --timeout-method thread -k "spill" > gpurun_out/r06_spill_t.log 2>&1; rc=$?; tail -3 gpurun_out/r06_spill_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/r06_ab.sh gpurun_out/r06_ab2 1 3 r5: d0:spill=0 d380:spill=380 d430:spill=430 d480:spill=480 r5b: d0b:spill=0
