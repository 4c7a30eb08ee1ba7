"""Small-batch decode workload for rocprofv3 (the restore path's kernels): LZ4 and zlib
decompression of 1 / 64 / 512 resident 16 KiB pages, 20 calls each, in one process.
    rocprofv3 --kernel-trace --stats -d DIR -o small -- python3 tools/run_small.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

plen = 16384
pages = codec.pagegen(512, plen, dist=0)
for cid in (1, 2):   # LZ4, zlib
    comp, clen = codec.compress_pages(pages, compressor_id=cid)
    torch.cuda.synchronize()
    for n in (1, 64, 512):
        c, l = comp[:n].contiguous(), clen[:n].contiguous()
        mx = int(l.max())
        out, rv = codec.decompress_pages(c, l, plen, compressor_id=cid, max_comp_len=mx)
        for _ in range(20):
            codec.decompress_pages(c, l, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx)
        torch.cuda.synchronize()
        assert bool((rv == plen).all()) and torch.equal(out, pages[:n])
print("ok")
