#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_zlib.py -x -q --timeout 120 --timeout-method thread > $OUT/p4_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p4_tests.log; exit 1; }
tail -1 $OUT/p4_tests.log
TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so timeout -k 10 200 python tools/zpar_pages.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/time_zlib.py 2>&1 | grep -v amdgpu.ids
TYCHE_ZLIB_PAR=0 timeout -k 10 200 python tools/time_zlib.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 tools/bin/cycle 65536 64 2000 16
echo DONE
