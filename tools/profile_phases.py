"""Diagnostic: per-phase cycle shares of the LZ4 decode kernel (profile build).

    python tyche_amd/_build.py --profile
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so python tools/profile_phases.py
Shares only (the stamps serialize the kernel a little); never quote its run time.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

NAMES = {1: "stage_in", 2: "parse_walk", 3: "parse_bridge", 5: "parse_compact", 6: "batch_decode",
         7: "literals", 8: "matches", 13: "decode_total", 12: "stage_out"}


def main():
    lib = _lib.load()
    prof = lib.tyche_debug_decode_profile
    prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    n = int(os.environ.get("PAGES", "65536"))
    plen = int(os.environ.get("PLEN", "16384"))
    dist = int(os.environ.get("DIST", "0"))
    pages = codec.pagegen(n, plen, dist=dist)
    comp, clen = codec.compress_pages(pages)
    torch.cuda.synchronize()
    mx = int(clen.max())
    buf = (ctypes.c_ulonglong * 16)()
    prof(buf, 1)
    out, rv = codec.decompress_pages(comp, clen, plen, max_comp_len=mx)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)
    prof(buf, 0)
    v = list(buf)
    pg = max(v[0], 1)
    tot = sum(v[k] for k in (1, 2, 3, 5, 6, 7, 8, 12))
    print(f"pages {v[0]}  seq/page {v[11] / pg:.0f}  hand-offs/page {v[4] / pg:.2f}  batches/page {v[10] / pg:.1f}"
          f"  groups/page {v[9] / pg:.0f}  ready/round {v[14] / max(v[9], 1):.2f}  max_comp {mx}")
    for k in (1, 2, 3, 5, 6, 7, 8, 12):
        print(f"  {NAMES[k]:14s} {v[k] / pg:10.0f} cyc/page  {100.0 * v[k] / tot:5.1f}%")


if __name__ == "__main__":
    main()
