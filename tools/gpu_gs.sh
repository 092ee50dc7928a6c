set -o pipefail
mkdir -p gpurun_out/gs
timeout -k 10 200 python -u tools/mb_gen_stamps.py 99 8 > gpurun_out/gs/g.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/gs/g.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/gs/g.txt
