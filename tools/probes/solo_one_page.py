"""Diagnostic driver for counter passes: decodes one 16 KiB LZ4 page N times (single-page decoder).

    rocprofv3 --pmc SQ_INSTS_VALU ... -- python tools/probes/solo_one_page.py [N]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tyche_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
pages = codec.pagegen(1, 16384, dist=0)
comp, clen = codec.compress_pages(pages)
mx = int(clen.max())
out, rv = codec.decompress_pages(comp, clen, 16384, max_comp_len=mx)
for _ in range(n):
    codec.decompress_pages(comp, clen, 16384, out=out, rv=rv, max_comp_len=mx)
torch.cuda.synchronize()
assert torch.equal(out, pages) and int(rv[0]) == 16384
print("ok", n)
