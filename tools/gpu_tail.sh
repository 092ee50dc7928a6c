set -o pipefail
mkdir -p gpurun_out/tail
timeout -k 10 200 python -u tools/mb_tail_c3.py > gpurun_out/tail/t.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/tail/t.txt; exit 1; }
grep -v amdgpu gpurun_out/tail/t.txt
