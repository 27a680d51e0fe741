# PMC passes for the system-tile kernels (and every other class) of the config-2 bench: texture
# address / data units, the vector L1, L2 hits, LDS -- one rocprofv3 --pmc run per hardware block
# group (never more than the block's counter slots), summarised per kernel by tools/pmc_summary.py.
#   usage: bash tools/pmc_systiles.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; TAG=${1:-dev}
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
i=0; csvs=""
for set in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $O/pmcx${i}_$TAG -o pmc --output-format csv -- $B > $O/pmcx${i}_$TAG.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmcx${i}_$TAG.log; exit 1; }
  csvs="$csvs $(find $O/pmcx${i}_$TAG -name '*counter_collection.csv' | head -1)"
done
python3 $R/tools/pmc_summary.py $O/pmc_systiles_$TAG.json $csvs
