#!/bin/bash
# SQ counters of the zstd decode kernels (two passes of 8)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/p14a -o run -- python tools/zstd_decode_once.py > $OUT/p14a.log 2>&1 || { echo PASS_A_FAILED; tail -5 $OUT/p14a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p14b -o run -- python tools/zstd_decode_once.py > $OUT/p14b.log 2>&1 || { echo PASS_B_FAILED; tail -5 $OUT/p14b.log; exit 1; }
grep -h "^ok\|MISMATCH" $OUT/p14a.log $OUT/p14b.log
echo DONE
