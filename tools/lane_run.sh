# A/B of the lane-per-page LZ4 decoders (lz4_decode_lane.hip) on the GPU box:
# LZ4 parity suite with every batch forced onto each variant (ring:window:linebuf),
# then decode timing.  RUNS / CFGS override the variant lists.
set -o pipefail
mkdir -p gpurun_out
export PAGES=${PAGES:-1048576}
for cfg in ${RUNS:-256:16:0 192:16:1}; do
IFS=: read ring win lb <<< "$cfg"
TYCHE_LZ4_LANE_RING=$ring TYCHE_LZ4_LANE_WIN=$win TYCHE_LZ4_LANE_LB=${lb:-0} TYCHE_LZ4_LANE_MIN=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_restore_queue.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lane_tests_${cfg//:/_}.log 2>&1 || { echo TESTS_FAILED $cfg; tail -30 gpurun_out/lane_tests_${cfg//:/_}.log; exit 1; }
echo $cfg; tail -1 gpurun_out/lane_tests_${cfg//:/_}.log
done
for cfg in ${CFGS:-256:16:0 128:16:1 192:16:1 224:16:1 256:16:1}; do
IFS=: read ring win lb <<< "$cfg"
echo ring:win:lb=$cfg; TYCHE_LZ4_LANE_RING=$ring TYCHE_LZ4_LANE_WIN=$win TYCHE_LZ4_LANE_LB=${lb:-0} timeout -k 10 200 python tools/time_decode.py 2>&1 | tail -1 || exit 1; done
