#!/bin/bash
# SQ counter passes over tools/run_codec.py (each its own rocprofv3 --pmc run, <= 8 SQ counters).
#   bash tools/pmc_enc.sh <out-prefix>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=${1:-pmc_enc}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export PAGES=${PAGES:-65536} REPS=1
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/${P}_$i -o run \
      -- python3 $R/tools/run_codec.py > $R/gpurun_out/${P}_$i.log 2>&1
done
echo done
