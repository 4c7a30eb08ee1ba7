#!/bin/bash
# A/B of the host path: tools/oldlib (an older build) vs the tree's library on the same box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for v in new old new old; do
  if [ $v = old ]; then export LD_LIBRARY_PATH=$R/tools/oldlib TYCHE_CODEC_LIB=$R/tools/oldlib/libtyche_codec.so; else unset LD_LIBRARY_PATH TYCHE_CODEC_LIB; fi
  timeout -k 10 120 tools/bin/latency 20 > $OUT/ab_lat_$v.jsonl || exit 1
  echo "$v latency:"; grep '"lz4", "page_len": 16384' $OUT/ab_lat_$v.jsonl | cut -c1-160
  timeout -k 10 200 python -c "
import sys, torch; sys.path.insert(0, '.')
import bench
from tyche_amd import codec
p = codec.pagegen(32768, 16384, dist=0)
torch.cuda.synchronize()
print('$v e2e', bench.e2e_host(p, 32768))
" 2>&1 | grep e2e || exit 1
done
echo DONE
