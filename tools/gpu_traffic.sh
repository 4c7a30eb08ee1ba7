#!/bin/bash
# HBM traffic of the bench kernels at the bench's sizes (C2: LZ4 1M x 16 KiB; C3: zstd 1M x 32 KiB;
# C4 shard: LZ4 1M x 8 KiB): a read pass and a WRITE_SIZE pass (separate rocprofv3 --pmc runs) over
# tools/run_codec.py with REPS=1, reduced by tools/pmc_traffic.py.  The read pass ("rdreq", round 6)
# takes the L2's memory-side read-request counters: TCC_EA0_RDREQ_DRAM_32B_sum counts 32-byte units
# with a 128-byte request as 4, beside TCC_EA0_RDREQ_sum, TCC_BUBBLE_sum and TCC_EA0_RDREQ_32B_sum
# (PASSES="FETCH_SIZE WRITE_SIZE" for the old pair).
#   bash tools/gpu_traffic.sh <round-tag, e.g. r02>
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r02}
mkdir -p $R/gpurun_out/traffic_$T
cd /tmp && export TMPDIR=/tmp REPS=1
run() {   # tag codec plen pages
  for c in ${PASSES:-rdreq WRITE_SIZE}; do
    [ "$c" = rdreq ] && pmc="TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum" || pmc=$c
    CODEC=$2 PLEN=$3 PAGES=$4 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv \
      -d $R/gpurun_out/traffic_$T/$1_$c -o run -- python3 $R/tools/run_codec.py > $R/gpurun_out/traffic_$T/$1_$c.log 2>&1 || { echo "pass $1 $c failed"; return 1; }
  done
}
run c2 lz4 16384 1048576 && run c3 zstd 32768 1048576 && run c4 lz4 8192 1048576 && echo done
