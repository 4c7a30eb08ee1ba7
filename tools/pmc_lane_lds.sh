#!/bin/bash
# LDS-side SQ counters of the lane LZ4 decoder and the encoders (one rocprofv3 --pmc pass, <= 8 SQ counters).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp PAGES=262144 REPS=1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT \
  --output-format csv -d $R/gpurun_out/pmc_lds -o run -- python3 $R/tools/run_codec.py > $R/gpurun_out/pmc_lds.log 2>&1 || echo "pass failed"
echo done
