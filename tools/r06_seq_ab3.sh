# Round 6: sequential-sum chunk per LDS round trip (16 default; variants 8 and 32) and the parallel method, alternating
set -o pipefail
bash tools/r06_ab.sh gpurun_out/r06_seq3_c3 2 3 par:seq_sum=0 def: v_seq32: v_seq8: || exit 1
EXTRA="--shard-of 8" bash tools/r06_ab.sh gpurun_out/r06_seq3_c5s8 1 5 par:seq_sum=0 def: v_seq32: || exit 1
EXTRA="--shard-of 16" bash tools/r06_ab.sh gpurun_out/r06_seq3_c5s16 1 5 par:seq_sum=0 def: v_seq32: || exit 1
bash tools/r06_ab.sh gpurun_out/r06_seq3_c5 1 5 par:seq_sum=0 def: v_seq32: || exit 1
