# Round evidence: bench line, rocprofv3 kernel-trace summary and PMC traffic.
# Usage (on the GPU box): bash tools/profile_round.sh r01
set -o pipefail
R=${1:-r01}
mkdir -p gpurun_out/$R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python bench.py --steps 100 --warmup 5 --no-cpu-baseline --profile-steps 10"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/kt -o bench -- $B > gpurun_out/$R/kt_bench.json 2> gpurun_out/$R/kt.err || { echo "kernel-trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$R/fetch -o p -- $B > /dev/null 2> gpurun_out/$R/fetch.err || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$R/write -o p -- $B > /dev/null 2> gpurun_out/$R/write.err || { echo "pmc write failed"; exit 1; }
python tools/pmc_traffic.py gpurun_out/$R/fetch gpurun_out/$R/write gpurun_out/$R/pmc_traffic.json > /dev/null
cp gpurun_out/$R/pmc_traffic.json profiles/${R}_pmc_traffic.json
timeout -k 10 300 python bench.py > gpurun_out/$R/bench.json 2> gpurun_out/$R/bench.err || { echo "bench failed"; exit 1; }
echo profile done
