mkdir -p gpurun_out
run() { echo "== $1"; env $1 timeout -k 10 200 python -u tools/diag_fused2.py 24 1 1 > gpurun_out/d3.log 2>&1 || { tail -5 gpurun_out/d3.log; return 1; }; grep -E "arrive nonzero after|differs" gpurun_out/d3.log; }
run "DIAG_GRAPH=0" && run "DIAG_SA_FUSED=0" && run "DIAG_SA_GROUPS=1" && run "DIAG_SA_GROUPS=2"
