#!/bin/bash
# Full GPU suite + smoke (what the driver runs at round end), one process each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/full_gpu.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 $OUT/full_gpu.log; exit 1; }
tail -2 $OUT/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
echo DONE
