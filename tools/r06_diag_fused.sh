set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_fused.py 3 30 1 > gpurun_out/diag_fused_c3.log 2>&1; echo "diag rc=$?"; tail -15 gpurun_out/diag_fused_c3.log
