set -o pipefail
mkdir -p gpurun_out/heavy
timeout -k 10 200 python -u tools/mb_frontier_heavy.py slots > gpurun_out/heavy/s.txt 2>&1 || { echo FAIL1; tail gpurun_out/heavy/s.txt; exit 1; }
grep -v amdgpu gpurun_out/heavy/s.txt
timeout -k 10 200 python -u tools/mb_frontier_heavy.py time > gpurun_out/heavy/t.txt 2>&1 || { echo FAIL2; tail gpurun_out/heavy/t.txt; exit 1; }
grep -v amdgpu gpurun_out/heavy/t.txt
