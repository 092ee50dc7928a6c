#!/bin/bash
# rocprofv3 kernel-trace stats of the driver's default command (python bench.py, 100 generations),
# plus the timed-window means (tools/kt_window.py, warmup 5, steps 100)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06prof_default
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o k -- python bench.py > $O/bench.json 2> $O/kt.err || { tail -5 $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/kt -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
python tools/kt_window.py $O/kernel_trace.csv 5 100 > $O/kernel_window.txt
cut -c1-60,90- $O/kernel_window.txt
head -4 $O/kernel_stats.csv | cut -c1-200
