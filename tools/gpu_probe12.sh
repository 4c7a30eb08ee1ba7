#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py -x -q --timeout 120 --timeout-method thread > $OUT/p12_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p12_tests.log; exit 1; }
tail -1 $OUT/p12_tests.log
PAGES=1048576 TYCHE_LIBS=tyche_amd/libtyche_codec_lit_lane1024.so,tyche_amd/libtyche_codec_lit_lane16.so,tyche_amd/libtyche_codec.so,tyche_amd/libtyche_codec_lit_lane4.so timeout -k 10 400 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
PLEN=8192 PAGES=1048576 TYCHE_LIBS=tyche_amd/libtyche_codec_lit_lane1024.so,tyche_amd/libtyche_codec.so timeout -k 10 400 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
echo DONE
