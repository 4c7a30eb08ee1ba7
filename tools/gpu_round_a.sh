#!/bin/bash
# Round measurement, part 1: the bench line and the kernel trace of the same workload.
set -e
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
tail -c 300 $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench \
    -- python3 $R/bench.py --no-cpu --e2e-pages 0 > $OUT/prof_bench_$TAG.log 2>&1
echo DONE
