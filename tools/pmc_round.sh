#!/bin/bash
# The round's counter passes over tools/run_codec.py (REPS=1: encode runs twice, decode once), one
# rocprofv3 --pmc run per counter set, within the per-block limits (<= 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD).
# Reduced by tools/pmc_round.py into profiles/<tag>_pmc_*.json (with the kernel-source digest).
#   bash tools/pmc_round.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04}
O=$R/gpurun_out/pmc_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp REPS=1 PAGES=${PAGES:-262144}
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 $R/tools/run_codec.py \
    > $O/$name.log 2>&1 || { echo "pass $name failed"; return 1; }
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU && \
pass sq2 SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH && \
pass lds SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE && \
pass tatd TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE && \
pass tcp TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE && \
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE && echo done
