#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py tests/test_c1_app.py -x -q --timeout 120 --timeout-method thread > $OUT/p8_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p8_tests.log; exit 1; }
tail -1 $OUT/p8_tests.log
TYCHE_LZ4_PARTS=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py -x -q --timeout 120 --timeout-method thread > $OUT/p8_tests2.log 2>&1 || { echo TESTS2_FAILED; tail -30 $OUT/p8_tests2.log; exit 1; }
tail -1 $OUT/p8_tests2.log
PAGES=1048576 TYCHE_LIBS=tyche_amd/libtyche_codec.so,tyche_amd/libtyche_codec_split3_a22_split3_b43.so,tyche_amd/libtyche_codec_split3_a26_split3_b45.so,tyche_amd/libtyche_codec_split3_a28_split3_b46.so timeout -k 10 400 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
TYCHE_LZ4_PARTS=2 PAGES=1048576 timeout -k 10 200 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
echo DONE
