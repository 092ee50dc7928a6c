# PMC evidence per bench config: HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
# and the SQ/GRBM counter groups of tools/pmc_counters.sh.
# Usage (on the GPU box): bash tools/r02_pmc.sh <round tag> <config>...
set -o pipefail
R=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$R
timeout -s KILL 60 rocprofv3 -L > gpurun_out/$R/counters_list.txt 2>&1 || true
for C in "$@"; do
  D=gpurun_out/$R/c$C
  mkdir -p $D
  B="bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline --profile-steps 3"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o p -- python $B > $D/fetch.log 2>&1 \
      || { echo "fetch pass c$C failed"; tail $D/fetch.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o p -- python $B > $D/write.log 2>&1 \
      || { echo "write pass c$C failed"; tail $D/write.log; exit 1; }
  python tools/pmc_traffic.py $D/fetch $D/write $D/pmc_traffic.json > /dev/null
  cp $D/pmc_traffic.json profiles/${R}_pmc_traffic_c$C.json
  bash tools/pmc_counters.sh $R/c$C --config $C --steps 10 --warmup 2 --no-cpu-baseline --profile-steps 3 \
      || { echo "counters c$C failed"; exit 1; }
  cp gpurun_out/$R/c$C/counters.json profiles/${R}_counters_c$C.json
  echo "c$C done"
done
