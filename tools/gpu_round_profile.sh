#!/bin/bash
# Round measurement on the GPU box: bench line, kernel-trace stats of the same
# workload, and the HBM PMC passes (FETCH_SIZE / WRITE_SIZE kept apart) for the
# C2 LZ4 kernels and the C3 zstd kernels.
# Usage (via gpurun): bash tools/gpu_round_profile.sh r01
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o bench \
    -- python3 $R/bench.py --no-cpu --e2e-pages 0 > $OUT/prof_bench_$TAG.log 2>&1
# reduce with tools/pmc_traffic.py (--calls lz4_decode=1: two size-class launches per call)
for spec in lz4:16384 zstd:32768; do
  c=${spec%%:*}; p=${spec##*:}
  export CODEC=$c PLEN=$p PAGES=262144 REPS=1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$TAG/${c}_fetch -o run \
      -- python3 $R/tools/run_codec.py > $OUT/pmc_fetch_${c}_$TAG.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$TAG/${c}_write -o run \
      -- python3 $R/tools/run_codec.py > $OUT/pmc_write_${c}_$TAG.log 2>&1
done
echo DONE
