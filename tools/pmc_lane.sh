#!/bin/bash
# PMC passes (each its own rocprofv3 --pmc run) over the FETCH_SIZE calibration probe and
# the LZ4 lane decoders (tools/run_codec.py, 262,144 x 16 KiB pages; LANE_MS=1 and 0).
#   bash tools/pmc_lane.sh <out-prefix>
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=${1:-pmc_lane}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export PAGES=262144 REPS=1
pass() {   # name, counters..., -- command
  local name=$1; shift
  local ctrs=""
  while [ "$1" != "--" ]; do ctrs="$ctrs $1"; shift; done; shift
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $R/gpurun_out/${P}_$name -o run -- "$@" > $R/gpurun_out/${P}_$name.log 2>&1 || echo "pass $name failed"
}
pass calib_fetch FETCH_SIZE -- $R/tools/bin/fetch_calib
pass calib_write WRITE_SIZE -- $R/tools/bin/fetch_calib
pass calib_req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- $R/tools/bin/fetch_calib
for ms in 1 0; do
  export TYCHE_LZ4_LANE_MS=$ms
  pass ms${ms}_fetch FETCH_SIZE -- python3 $R/tools/run_codec.py
  pass ms${ms}_write WRITE_SIZE -- python3 $R/tools/run_codec.py
  pass ms${ms}_req TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum -- python3 $R/tools/run_codec.py
  pass ms${ms}_sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -- python3 $R/tools/run_codec.py
done
echo done
