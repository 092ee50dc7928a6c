set -o pipefail
mkdir -p gpurun_out/sc3
TRAIN_ONLY=1 timeout -k 10 200 python -u tools/mb_scan3_stamps.py 512 > gpurun_out/sc3/s.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/sc3/s.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/sc3/s.txt
