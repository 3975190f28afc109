#!/bin/bash
# PMC passes over tools/prof_one.py for a set of K2 variants on one workload (tooling):
#   bash tools/pmc_variants.sh <tag> <workload> <variants> [bpc]
# writes gpurun_out/<tag>/p<i>_counter_collection.csv; summarise with tools/pmc_summary.py
set -o pipefail
TAG=$1; W=$2; VS=$3; BPC=${4:-0}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT|GRBM_GUI_ACTIVE FETCH_SIZE|WRITE_SIZE SQ_INSTS_VMEM_WR"
IFS='|' read -ra PS <<< "$P"; i=0
for c in "${PS[@]}"; do
  i=$((i+1))
  timeout -k 5 -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/$TAG -o p$i -- python3 tools/prof_one.py --workload $W --variants $VS --bpc $BPC > gpurun_out/$TAG.p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc-done
