# frontier timeline with packed-slot counts (stamped build), then config-4 profile refresh
set -o pipefail
mkdir -p gpurun_out/pack
TRAIN_ONLY=1 timeout -k 10 200 python -u tools/mb_frontier_timeline.py 512 > gpurun_out/pack/tl.txt 2>&1 || { echo TL_FAIL; tail -20 gpurun_out/pack/tl.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/pack/tl.txt
bash tools/r02_profile.sh r02f 4
