# A/B of the lane-per-page LZ4 decoders (lz4_decode_lane.hip) on the GPU box:
# LZ4 parity suite with every batch forced onto each variant (ring:window),
# then decode timing.  RUNS / CFGS override the variant lists.
set -o pipefail
mkdir -p gpurun_out
export PAGES=1048576
for cfg in ${RUNS:-256:32 256:16 0:32}; do
TYCHE_LZ4_LANE_RING=${cfg%%:*} TYCHE_LZ4_LANE_WIN=${cfg##*:} TYCHE_LZ4_LANE_MIN=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_restore_queue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lane_tests_${cfg/:/_}.log 2>&1 || { echo TESTS_FAILED $cfg; tail -30 gpurun_out/lane_tests_${cfg/:/_}.log; exit 1; }
echo $cfg; tail -1 gpurun_out/lane_tests_${cfg/:/_}.log
done
for cfg in ${CFGS:-256:32 256:16 128:16 512:16}; do echo ring:win=$cfg; TYCHE_LZ4_LANE_RING=${cfg%%:*} TYCHE_LZ4_LANE_WIN=${cfg##*:} timeout -k 10 200 python tools/time_decode.py 2>&1 | tail -1 || exit 1; done
