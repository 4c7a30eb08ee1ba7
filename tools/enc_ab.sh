# LZ4 encoder A/B: the parity suite on the default kernel, then 1M x 16 KiB and 8 KiB timings
# for the default (split) and the one-wave kernel (TYCHE_LZ4_ENC=1).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_host_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_ab_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/enc_ab_tests.log; exit 1; }
tail -1 gpurun_out/enc_ab_tests.log
for e in 0 1; do for pl in 16384 8192; do echo "ENC=$e PLEN=$pl"; TYCHE_LZ4_ENC=$e PLEN=$pl PAGES=1048576 timeout -k 10 200 python tools/time_variant.py 2>&1 | tail -1 || exit 1; done; done
