# config-2 tail phases (register-held stamps, no memory waits)
set -o pipefail
mkdir -p gpurun_out/sc2s
timeout -k 10 300 python -u tools/mb_scan2_stamps.py > gpurun_out/sc2s/c2_t.log 2>&1 || { cat gpurun_out/sc2s/c2_t.log; exit 1; }
grep -E "tail" gpurun_out/sc2s/c2_t.log
