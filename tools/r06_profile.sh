#!/bin/bash
# round 6 evidence for one workload: rocprofv3 kernel-trace stats, PMC traffic
# (FETCH_SIZE and WRITE_SIZE in separate passes) and SQ counters, plus the bench
# line.  Usage (on the GPU box): bash tools/r06_profile.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-steps 5 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- $B > $O/kt_bench.json 2> $O/kt.err || { tail -5 $O/kt.err; echo "kernel-trace failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- $B > /dev/null 2> $O/fetch.err || { tail -5 $O/fetch.err; echo "pmc fetch failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- $B > /dev/null 2> $O/write.err || { tail -5 $O/write.err; echo "pmc write failed"; exit 1; }
python tools/pmc_traffic.py $O/fetch $O/write $O/pmc_traffic.json > /dev/null
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o p -- $B > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/pmc_summary.py $O > $O/counters.json
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/kt -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
python tools/kt_window.py $O/kernel_trace.csv 5 20 > $O/kernel_window.txt
cat $O/kernel_window.txt | cut -c1-60,90-
python tools/bench_summary.py $O/kt_bench.json
head -5 $O/kernel_stats.csv | cut -c1-160
python - $O/pmc_traffic.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.get("kernels", {}).items():
    print(k, {kk: (round(vv / 1e6, 1) if isinstance(vv, (int, float)) and vv > 1e5 else vv) for kk, vv in v.items()})
PY
echo profile done
