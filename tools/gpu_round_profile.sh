#!/bin/bash
# Round measurement on the GPU box: the bench line, the kernel-trace stats of the same workload,
# the HBM PMC passes at the bench's sizes (tools/gpu_traffic.sh: FETCH_SIZE / WRITE_SIZE kept apart),
# every codec's rates on resident pages (tools/time_codecs.py), the Buffer-API latency table
# (tools/latency.c), the sweep/restore cycles (tools/cycle.c, tools/cycle_live.c) and the host path's
# link probe and stage clocks (tools/host_probe.py).
# Usage (via gpurun): bash tools/gpu_round_profile.sh r03
set -e
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
tail -c 300 $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench \
    -- python3 $R/bench.py --no-cpu --e2e-pages 0 > $OUT/prof_bench_$TAG.log 2>&1
cd $R
bash tools/gpu_traffic.sh $TAG
timeout -k 10 300 python tools/time_codecs.py > $OUT/time_codecs_$TAG.log 2>&1
timeout -k 10 120 tools/bin/latency 30 > $OUT/latency_$TAG.jsonl
timeout -k 10 200 tools/bin/cycle 65536 64 2000 16 > $OUT/cycle_$TAG.json
timeout -k 10 200 tools/bin/cycle_live 12000 64 600 16 10 > $OUT/cycle_live_$TAG.json
timeout -k 10 300 python tools/host_probe.py 65536 32,64 > $OUT/host_probe_$TAG.jsonl 2>&1
echo DONE
