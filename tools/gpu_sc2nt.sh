# config-2 scan phases with the tail-phase stamps compiled out (tail = stamp 4 -> 5 only)
set -o pipefail
mkdir -p gpurun_out/sc2s
STAMP_LIB=tools/mb/libsgmm_stamps_nt.so timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_nt.log 2>&1 || { cat gpurun_out/sc2s/c2_nt.log; exit 1; }
grep -vE "waves per|table|amdgpu.ids" gpurun_out/sc2s/c2_nt.log
