#!/bin/bash
# A/B of TYCHE_BRIDGE_STEPS (token-chain bridge steps per hand-off round): LZ4 jump / zlib jump timings
# (build the variants first: python -c "from tyche_amd import _build; [_build.build(defines=(f\"TYCHE_BRIDGE_STEPS={v}\",)) for v in (2, 8)]")
# per library build (tools/time_jump.py, batches 1..512).  Usage (via gpurun): bash tools/ab_bridge.sh
for lib in tyche_amd/libtyche_codec.so tyche_amd/libtyche_codec_bridge_steps2.so tyche_amd/libtyche_codec_bridge_steps8.so; do
  echo "== $lib"
  TYCHE_CODEC_LIB=$lib timeout -k 10 200 python tools/time_jump.py 2>&1 | grep -E '"(jump|zlib-jump-wg)"' | grep -E '"batch": (1|64|512),' | grep -v '"batch": 1[0-9]'
done
