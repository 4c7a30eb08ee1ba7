#!/bin/bash
# Round measurement, part 2: HBM PMC passes, every codec's rates, Buffer-API latency, sweep/restore cycle.
set -e
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
bash tools/gpu_traffic.sh $TAG
timeout -k 10 300 python tools/time_codecs.py > $OUT/time_codecs_$TAG.log 2>&1
timeout -k 10 120 tools/bin/latency 30 > $OUT/latency_$TAG.jsonl
timeout -k 10 200 tools/bin/cycle 65536 64 2000 16 > $OUT/cycle_$TAG.json
echo DONE
