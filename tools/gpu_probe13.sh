#!/bin/bash
# zstd split decode: new parity test + kernel trace of the C3 timing loop
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 200 --timeout-method thread -k "fused_kernel_and_chunked" > $OUT/p13_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p13_tests.log; exit 1; }
tail -1 $OUT/p13_tests.log
CODEC=zstd PLEN=32768 PAGES=65536 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p13prof -o run -- python tools/time_variant.py > $OUT/p13_tv.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/p13_tv.log; exit 1; }
grep -v amdgpu.ids $OUT/p13_tv.log | tail -2
find $OUT/p13prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -12
echo DONE
