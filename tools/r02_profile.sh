# Round-2 evidence for one bench config: rocprofv3 kernel-trace stats, PMC
# HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes), SQ counter groups,
# then the bench line itself (reads the new traffic summary).
# Usage (on the GPU box): bash tools/r02_profile.sh <tag> <config>
set -o pipefail
R=$1; C=$2
D=gpurun_out/$R/c$C
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --profile-steps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- python $B > $D/kt_bench.json 2> $D/kt.err \
    || { echo "kernel-trace failed"; tail $D/kt.err; exit 1; }
cp $(find $D/kt -name "*kernel_stats.csv" | head -1) $D/kernel_stats.csv
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o p -- python $B > $D/fetch.log 2>&1 \
    || { echo "fetch pass failed"; tail $D/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o p -- python $B > $D/write.log 2>&1 \
    || { echo "write pass failed"; tail $D/write.log; exit 1; }
python tools/pmc_traffic.py $D/fetch $D/write $D/pmc_traffic.json > /dev/null
bash tools/pmc_counters.sh $R/c$C --config $C --steps 20 --warmup 3 --no-cpu-baseline --profile-steps 5 \
    || { echo "counters failed"; exit 1; }
true
timeout -k 10 300 python bench.py --config $C > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail $D/bench.err; exit 1; }
true
echo "c$C profiled"
