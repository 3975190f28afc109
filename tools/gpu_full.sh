#!/bin/bash
# One GPU call: parity tests, headline bench, kernel trace, PMC passes (c2, c3), other configs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_round.sh all || exit $?
for w in ${PMC_WL:-c2 c3}; do
  OUT=gpurun_out/pmc_$w bash tools/pmc.sh "--workload $w" FETCH_SIZE WRITE_SIZE "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" || exit $?
done
OUT=gpurun_out/pmc_nat bash tools/pmc.sh "--nat 0" FETCH_SIZE WRITE_SIZE "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES" "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" || exit $?
bash tools/gpu_extra.sh
