"""Runs one compress + decompress pass over N synthetic pages (profiling target).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/run_codec.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

n = int(os.environ.get("PAGES", "262144"))
plen = int(os.environ.get("PLEN", "16384"))
reps = int(os.environ.get("REPS", "2"))
pages = codec.pagegen(n, plen, dist=int(os.environ.get("DIST", "0")))
comp, clen = codec.compress_pages(pages)
torch.cuda.synchronize()
mx = int(clen.max())
for _ in range(reps):
    codec.compress_pages(pages, out=comp, out_len=clen)
    out, rv = codec.decompress_pages(comp, clen, plen, max_comp_len=mx)
torch.cuda.synchronize()
assert bool((rv == plen).all()) and torch.equal(out, pages)
print("ok", n, plen, float(n * plen) / float(clen.sum()))
