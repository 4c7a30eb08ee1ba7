#!/bin/bash
# zlib lane-parallel inflate: GPU parity first, then latency / throughput, then the lane decoder's LDS counters.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_zlib.py -x -q --timeout 120 --timeout-method thread > $OUT/zpar_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/zpar_tests.log; exit 1; }
tail -2 $OUT/zpar_tests.log
timeout -k 10 120 tools/bin/latency 20 > $OUT/zpar_latency.jsonl && grep zlib $OUT/zpar_latency.jsonl
TYCHE_ZLIB_PAR=0 timeout -k 10 120 tools/bin/latency 20 > $OUT/zpar_latency_serial.jsonl && grep zlib $OUT/zpar_latency_serial.jsonl
timeout -k 10 200 python tools/time_zlib.py > $OUT/zpar_time.log 2>&1; tail -5 $OUT/zpar_time.log
TYCHE_ZLIB_PAR=0 timeout -k 10 200 python tools/time_zlib.py > $OUT/zpar_time_serial.log 2>&1; tail -5 $OUT/zpar_time_serial.log
timeout -k 10 200 tools/bin/cycle 65536 64 2000 16 > $OUT/zpar_cycle.json && cat $OUT/zpar_cycle.json
PAGES=1048576 TYCHE_LIBS=tyche_amd/libtyche_codec.so,tyche_amd/libtyche_codec_abl128.so,tyche_amd/libtyche_codec_abl64.so,tyche_amd/libtyche_codec_abl256.so timeout -k 10 400 python tools/time_variant.py > $OUT/lane_abl.log 2>&1; cat $OUT/lane_abl.log
bash tools/pmc_lane_lds.sh
echo DONE
