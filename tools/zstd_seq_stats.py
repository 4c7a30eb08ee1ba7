"""Writes zstd frames for tools/zstd_seq_stats.c (zlib streams for tools/zlib_sym_stats.c
with --codec zlib) as [u32 length][frame] ....

    python tools/zstd_seq_stats.py frames.npz out.bin     # device frames (tools/dump_frames.py)
    python tools/zstd_seq_stats.py --ref 2000 out.bin     # the reference's level-1 frames of bench pages
"""
import argparse
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("out")
ap.add_argument("--ref", type=int, default=0)
ap.add_argument("--plen", type=int, default=16384)
ap.add_argument("--codec", default="zstd")
a = ap.parse_args()
with open(a.out, "wb") as f:
    if a.ref:
        from oracle import oracle as O
        pages = O.pagegen(a.ref, a.plen, seed=11, dist=0)
        for i in range(a.ref):
            if a.codec == "zlib":
                fr = O.ref_zlib_compress(pages[i].tobytes(), 1)
            else:
                fr = O.ref_zstd_compress_blocks(pages[i].tobytes(), a.plen, 1)
            f.write(struct.pack("<I", len(fr)) + bytes(fr))
    else:
        z = np.load(a.src)
        for row, n in zip(z["comp"], z["clen"]):
            f.write(struct.pack("<I", int(n)) + row[:int(n)].tobytes())
