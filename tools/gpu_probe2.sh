#!/bin/bash
# zlib parallel-path diagnostics + a runtime trace of the Buffer-API latency run (host overhead breakdown).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python tools/zpar_probe.py > $OUT/zpar_probe.log 2>&1; cat $OUT/zpar_probe.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --runtime-trace --output-format csv -d $OUT/lat_trace -o lat -- $R/tools/bin/latency 5 > $OUT/lat_trace.log 2>&1 || echo "trace failed"
ls $OUT/lat_trace
echo DONE
