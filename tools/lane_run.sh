# A/B of the lane-per-page LZ4 decoder (lz4_decode_lane.hip) on the GPU box:
# LZ4 parity suite with every batch forced onto it, then decode timing.
set -o pipefail
mkdir -p gpurun_out
export PAGES=1048576
TYCHE_LZ4_LANE_MIN=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_restore_queue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lane_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/lane_tests.log; exit 1; }
tail -2 gpurun_out/lane_tests.log
for w in ${WAVES:-2 3 4 6 8}; do echo waves=$w; TYCHE_LZ4_LANE_WAVES=$w timeout -k 10 200 python tools/time_decode.py 2>&1 | tail -1 || exit 1; done
