# frontier timeline after packing (stamped build, config-3 training launch, all-whole default)
set -o pipefail
mkdir -p gpurun_out/tl3
TRAIN_ONLY=1 timeout -k 10 200 python -u tools/mb_frontier_timeline.py 512 > gpurun_out/tl3/tl.txt 2>&1 || { echo TL_FAIL; tail -20 gpurun_out/tl3/tl.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tl3/tl.txt
