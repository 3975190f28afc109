#!/bin/bash
# Where a kernel's time goes beyond HBM bytes (tooling): address translation (UTCL1), the TA / TCP
# pipeline stalls and the SQ's VMEM issue FIFOs, per config.  One --pmc pass per line (gfx950 slots:
# <= 4 TCP, 2 TA, 8 SQ).  usage: tools/pmc_deep.sh <tag> "<configs: c2 c3 c1 nat natprobe c3_64 c3_576 c3_1500>"
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03}; CFGS=${2:-"c2 c3 nat"}
P=("TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_UTCL1_STALL_MULTI_MISS"
   "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"
   "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES"
   "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES SQ_WAVES")
for w in $CFGS; do
  case $w in
    nat) args="--nat 0 --nat-mask 15";;
    natprobe) args="--nat 0 --nat-mask 15 --nat-probe";;
    c3_*) args="--workload c3 --class-len ${w#c3_}";;   # one C3 size class alone
    *) args="--workload $w";;
  esac
  i=0
  for c in "${P[@]}"; do
    i=$((i+1))
    echo "=== $w p$i $(date +%T)"
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_deep_$w -o p$i -- python3 tools/prof_one.py $args > gpurun_out/${TAG}_deep_${w}_p$i.log 2>&1
    rc=$?; echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_deep_${w}_p$i.log; exit $rc; fi
  done
done
echo ALLDONE
