# frontier phase stamps + shader clock: one wave per SIMD vs the config-3 residency
set -o pipefail
mkdir -p gpurun_out/ph2
for P in 512 2560; do
  TRAIN_ONLY=1 timeout -k 10 200 python -u tools/mb_frontier_stamps.py $P 0.05 > gpurun_out/ph2/phase_$P.txt 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/ph2/phase_$P.txt; exit 1; }
  echo "P=$P"; grep -v amdgpu.ids gpurun_out/ph2/phase_$P.txt
done
