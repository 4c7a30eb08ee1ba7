# A/B of the lane-per-page LZ4 decoders (lz4_decode_lane.hip) on the GPU box:
# LZ4 parity suite with every batch forced onto them, then decode timing.
set -o pipefail
mkdir -p gpurun_out
export PAGES=1048576
for ring in 1 0; do
TYCHE_LZ4_LANE_RING=$ring TYCHE_LZ4_LANE_MIN=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_restore_queue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lane_tests_$ring.log 2>&1 || { echo TESTS_FAILED ring=$ring; tail -30 gpurun_out/lane_tests_$ring.log; exit 1; }
tail -1 gpurun_out/lane_tests_$ring.log
done
for cfg in ${CFGS:-1:4 1:3 1:2 0:4}; do echo ring:waves=$cfg; TYCHE_LZ4_LANE_RING=${cfg%%:*} TYCHE_LZ4_LANE_WAVES=${cfg##*:} timeout -k 10 200 python tools/time_decode.py 2>&1 | tail -1 || exit 1; done
