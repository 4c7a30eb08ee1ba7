#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TYCHE_LZ4_LANE_MIN=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py -x -q --timeout 120 --timeout-method thread > $OUT/p6_lane_tests.log 2>&1 || { echo LANE_TESTS_FAILED; tail -30 $OUT/p6_lane_tests.log; exit 1; }
tail -1 $OUT/p6_lane_tests.log
PAGES=1048576 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
TYCHE_LZ4_COOP=0 PAGES=1048576 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
echo DONE
