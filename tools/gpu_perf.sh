set -o pipefail
timeout -k 10 300 python tools/mb_rollout.py 3600 16 > gpurun_out/mb_16.json 2> gpurun_out/mb.err || exit 1
timeout -k 10 300 python tools/mb_rollout.py 3600 32 > gpurun_out/mb_32.json 2>> gpurun_out/mb.err || exit 1
bash tools/pmc.sh
