# occupancy probe: device properties; table waves per CU at start with HP = 16 (LDS 26.7 KB) vs HP = 20
set -o pipefail
mkdir -p gpurun_out/sc2s
timeout -k 10 120 python -u tools/devattr.py || exit 1
STAMP_LIB=tools/mb/libsgmm_stamps_hp16.so STAMP_OUT=gpurun_out/sc2s/c2_hp16.npz timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_hp16.log 2>&1 || { cat gpurun_out/sc2s/c2_hp16.log; exit 1; }
grep -E "table|waves per" gpurun_out/sc2s/c2_hp16.log
