# config-2 scan / table phase stamps (stamped libraries: 4 and 5 table waves per SIMD)
set -o pipefail
mkdir -p gpurun_out/sc2s
STAMP_OUT=gpurun_out/sc2s/c2.npz timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2.log 2>&1 || { cat gpurun_out/sc2s/c2.log; exit 1; }
cat gpurun_out/sc2s/c2.log
STAMP_OUT=gpurun_out/sc2s/c2_5.npz STAMP_LIB=tools/mb/libsgmm_stamps5.so timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_5.log 2>&1 || { cat gpurun_out/sc2s/c2_5.log; exit 1; }
cat gpurun_out/sc2s/c2_5.log
