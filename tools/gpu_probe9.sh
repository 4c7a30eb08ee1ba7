#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_zlib.py tests/test_host_engine.py -x -q --timeout 120 --timeout-method thread > $OUT/p9_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p9_tests.log; exit 1; }
tail -1 $OUT/p9_tests.log
for pl in 8192 16384 32768; do
CODEC=zlib PLEN=$pl PAGES=131072 timeout -k 10 400 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
done
timeout -k 10 200 python tools/time_zlib.py 2>&1 | grep -v amdgpu.ids
echo DONE
