set -o pipefail
mkdir -p gpurun_out/kt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt/run -o kt -- python bench.py --steps 60 --warmup 5 --no-cpu-baseline --profile-steps 2 > gpurun_out/kt/bench.json 2> gpurun_out/kt/err.log || { echo KT_FAIL; tail gpurun_out/kt/err.log; exit 1; }
python tools/kt_timeline.py $(ls gpurun_out/kt/run/*kernel_trace.csv | head -1) 40
