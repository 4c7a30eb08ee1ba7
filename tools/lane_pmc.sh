# PMC passes over the LZ4 codec pair (tools/run_codec.py, 256K x 16 KiB pages):
# HBM bytes (FETCH_SIZE, WRITE_SIZE) and L2 hit/miss, one counter set per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/lanepmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export CODEC=lz4 PLEN=16384 PAGES=262144 REPS=1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/run_codec.py > $OUT/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo DONE
