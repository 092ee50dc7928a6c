# Instruction mix of one kernel in a gfx950 assembly file.
# Usage: bash tools/isa_stats.sh <file.s> <kernel-name-substring> [out.s]
S=$1; K=$2; O=${3:-/tmp/k.s}
L=$(grep -n "^_Z[^ ]*$K[^ ]*:" "$S" | head -1 | cut -d: -f1)
[ -z "$L" ] && { echo "no kernel $K"; exit 1; }
awk -v L="$L" 'NR>=L{print} NR>L && /^\.Lfunc_end/{exit}' "$S" > "$O"
echo "$K: $(wc -l < "$O") lines"
for p in v_mfma ds_read ds_write v_pk_fma 'v_fma_f32\|v_fmac_f32' v_max_i32 accvgpr s_nop scratch _f64 s_waitcnt v_cndmask; do echo -n "$p=$(grep -c "$p" "$O") "; done; echo
grep -A40 "\.name:.*$K" "$S" | grep -m4 'vgpr_count\|sgpr_count\|spill'
grep -B40 "\.name:.*$K" "$S" | grep 'group_segment_fixed_size\|agpr_count' | tail -2
