"""Diagnostic: one zstd decode of PAGES x PLEN synthetic pages (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

n = int(os.environ.get("PAGES", "16384"))
plen = int(os.environ.get("PLEN", "32768"))
pages = codec.pagegen(n, plen, dist=0)
comp, clen = codec.compress_pages(pages, compressor_id=3)
torch.cuda.synchronize()
out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=3, max_comp_len=int(clen.max()))
torch.cuda.synchronize()
print("ok" if bool((rv == plen).all()) and torch.equal(out, pages) else "MISMATCH", "max_comp", int(clen.max()))
