"""Runs one compress + decompress pass over N synthetic pages (profiling target).

    CODEC=lz4|zstd|zlib PLEN=16384 PAGES=262144 \
        rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/run_codec.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

IDS = {"lz4": 1, "zlib": 2, "zstd": 3}
cid = IDS[os.environ.get("CODEC", "lz4")]
n = int(os.environ.get("PAGES", "262144"))
plen = int(os.environ.get("PLEN", "16384"))
reps = int(os.environ.get("REPS", "2"))
pages = codec.pagegen(n, plen, dist=int(os.environ.get("DIST", "0")))
comp, clen = codec.compress_pages(pages, compressor_id=cid)
torch.cuda.synchronize()
mx = int(clen.max())
for _ in range(reps):
    codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen)
    out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=cid, max_comp_len=mx)
torch.cuda.synchronize()
assert bool((rv == plen).all()) and torch.equal(out, pages)
print("ok", os.environ.get("CODEC", "lz4"), n, plen, float(n * plen) / float(clen.sum()))
