"""Writes device-encoded frames of bench pages to an npz (for tools/zstd_frame_stats.py).

    CODEC=zstd PLEN=16384 PAGES=64 python tools/dump_frames.py gpurun_out/frames.npz
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

IDS = {"lz4": 1, "zlib": 2, "zstd": 3}
n = int(os.environ.get("PAGES", "64"))
plen = int(os.environ.get("PLEN", "16384"))
pages = codec.pagegen(n, plen, seed=int(os.environ.get("SEED", "11")), first=int(os.environ.get("FIRST", "0")),
                      dist=int(os.environ.get("DIST", "0")))
comp, clen = codec.compress_pages(pages, compressor_id=IDS[os.environ.get("CODEC", "zstd")])
torch.cuda.synchronize()
np.savez(sys.argv[1], comp=comp.cpu().numpy(), clen=clen.cpu().numpy())
print("ratio", n * plen / float(clen.sum()))
