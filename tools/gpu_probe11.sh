#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export TYCHE_LZ4_WRITER=1
# small first: one launch of 64K pages under a short limit (a protocol deadlock must not hang the box)
PAGES=65536 timeout -k 5 60 python tools/time_variant.py > $OUT/p11_small.log 2>&1 || { echo SMALL_FAILED; tail -5 $OUT/p11_small.log; exit 1; }
grep -v amdgpu.ids $OUT/p11_small.log
TYCHE_LZ4_LANE_MIN=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py -x -q --timeout 60 --timeout-method thread > $OUT/p11_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p11_tests.log; exit 1; }
tail -1 $OUT/p11_tests.log
PAGES=1048576 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
TYCHE_LZ4_WRITER=0 PAGES=1048576 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
echo DONE
