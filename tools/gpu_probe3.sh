#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_zlib.py tests/test_restore_queue.py tests/test_host_engine.py tests/test_gpu_lz4.py -x -q --timeout 120 --timeout-method thread > $OUT/p3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/p3_tests.log; exit 1; }
tail -2 $OUT/p3_tests.log
TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so timeout -k 10 200 python tools/zpar_pages.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 tools/bin/latency 20 > $OUT/p3_latency.jsonl && cat $OUT/p3_latency.jsonl
timeout -k 10 200 tools/bin/cycle 65536 64 2000 16 > $OUT/p3_cycle.json && cat $OUT/p3_cycle.json
echo DONE
