# cross-wave MFMA/VALU issue microbenchmark + frontier phase stamps (training-only launch)
set -o pipefail
mkdir -p gpurun_out/mb2
timeout -k 10 120 ./tools/mb/mb_mfma_xwave2 > gpurun_out/mb2/xwave2.txt 2>&1 || { echo MB_FAIL; cat gpurun_out/mb2/xwave2.txt; exit 1; }
cat gpurun_out/mb2/xwave2.txt
TRAIN_ONLY=1 timeout -k 10 200 python -u tools/mb_frontier_stamps.py 512 0.05 > gpurun_out/mb2/phase_train.txt 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/mb2/phase_train.txt; exit 1; }
cat gpurun_out/mb2/phase_train.txt
