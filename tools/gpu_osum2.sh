set -o pipefail
for v in v2 v1; do SGMM_SCAN=$v timeout -k 10 120 python -u tools/mb_osum2.py 2>&1 | grep -v amdgpu.ids || exit 1; done
SGMM_LIB=tools/mb/libsgmm_stamps.so timeout -k 10 120 python -u tools/mb_osum2.py 2>&1 | grep -v amdgpu.ids || exit 1
SGMM_LIB=tools/mb/libsgmm_stamps.so timeout -k 10 200 python -u tools/mb_scan2_stamps.py 2>&1 | grep -v amdgpu.ids
