#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > $OUT/p10_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p10_tests.log; exit 1; }
tail -1 $OUT/p10_tests.log
for pl in 32768 16384; do
CODEC=zstd PLEN=$pl PAGES=65536 timeout -k 10 400 python tools/time_variant.py 2>&1 | grep -v amdgpu.ids
done
TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so timeout -k 10 200 python tools/zstd_prof.py 2>&1 | grep -v amdgpu.ids
echo DONE
