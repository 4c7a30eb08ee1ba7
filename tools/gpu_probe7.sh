#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > $OUT/p7_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p7_tests.log; exit 1; }
tail -1 $OUT/p7_tests.log
CODEC=zstd PLEN=32768 PAGES=262144 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
CODEC=zstd PLEN=16384 PAGES=262144 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
echo DONE
