# Round 6: the pipelined sequential sum (default rule) against the parallel method, alternating
set -o pipefail
bash tools/r06_ab.sh gpurun_out/r06_seq2_c3 2 3 par:seq_sum=0 def: || exit 1
EXTRA="--shard-of 16" bash tools/r06_ab.sh gpurun_out/r06_seq2_c5s16 1 5 par:seq_sum=0 def: w64:scan_threads=64 || exit 1
EXTRA="--shard-of 8" bash tools/r06_ab.sh gpurun_out/r06_seq2_c5s8 1 5 par:seq_sum=0 def: || exit 1
bash tools/r06_ab.sh gpurun_out/r06_seq2_c5 1 5 par:seq_sum=0 def: || exit 1
bash tools/r06_ab.sh gpurun_out/r06_seq2_c2 1 2 par: seq:seq_sum=1 || exit 1
