#!/bin/bash
# SQ counter pass over tools/run_codec.py (one rocprofv3 --pmc run, <= 8 SQ counters).
#   bash tools/pmc_sq.sh <out-subdir> [counters...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
SUB=${1:-pmc_sq}; shift || true
CTRS=${@:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export PAGES=${PAGES:-65536} REPS=1
timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/$SUB -o run \
    -- python3 $R/tools/run_codec.py > $R/gpurun_out/$SUB.log 2>&1
echo done
