"""Diagnostic: sha1 of a codec's compressed streams (and their total bytes) over synthetic pages, so
that two library builds can be checked for byte-identical encoder output:

    CODEC=zstd PLEN=32768 PAGES=65536 TYCHE_CODEC_LIB=... python tools/stream_digest.py
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

cid = _lib.COMPRESSOR_IDS[os.environ.get("CODEC", "zstd")]
plen = int(os.environ.get("PLEN", "32768"))
n = int(os.environ.get("PAGES", "65536"))
dev = torch.device("cuda:0")
out = {"lib": os.path.basename(_lib.LIB_PATH), "codec": os.environ.get("CODEC", "zstd"), "plen": plen, "pages": n}
for dist in range(6):
    pages = codec.pagegen(n, plen, dist=dist, first=dist * 7, device=dev)
    comp, clen = codec.compress_pages(pages, compressor_id=cid)
    torch.cuda.synchronize()
    h = hashlib.sha1()
    cl = clen.cpu().numpy()
    cc = comp.cpu().numpy()
    for i in range(n):
        h.update(cc[i, :cl[i]].tobytes())
    out[f"dist{dist}"] = {"bytes": int(cl.sum()), "sha1": h.hexdigest()[:16]}
print(json.dumps(out), flush=True)
