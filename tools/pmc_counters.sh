# SQ/GRBM counter passes over a short bench run, one counter group per
# rocprofv3 run (no trace domains with --pmc), for the table kernel's bound.
# Usage (on the GPU box): bash tools/pmc_counters.sh <tag> <bench args...>
# Output: gpurun_out/<tag>/pmc_<i>/ and gpurun_out/<tag>/counters.json
set -o pipefail
TAG=$1
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/$TAG/pmc_$i -o p -- python bench.py "$@" \
      > gpurun_out/$TAG/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/counters.json
echo pmc done
