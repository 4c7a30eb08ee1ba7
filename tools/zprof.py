"""Diagnostic: phase shares of the lane-parallel zlib inflate (profile build).

    python -c "import tyche_amd._build as b; b.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so python tools/zprof.py
Cycles are clock64() deltas of lane 0 summed over pages (the stamps serialize a little)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

NAMES = {1: "header+tables", 2: "walk", 3: "bridge+handoffs", 4: "count", 5: "write", 7: "block end",
         6: "matches", 8: "adler"}


def run(n, plen):
    lib = _lib.load()
    prof = lib.tyche_debug_zlib_profile
    prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    pages = codec.pagegen(max(n, 64), plen, dist=0)[:n].contiguous()
    comp, clen = codec.compress_pages(pages, compressor_id=2)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 16)()
    prof(buf, 1)
    out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=2, max_comp_len=int(clen.max()))
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)
    prof(buf, 0)
    v = list(buf)
    pg = max(v[0], 1)
    tot = sum(v[k] for k in NAMES)
    print(f"n={n} plen={plen}: pages {v[0]}  cycles/page {tot / pg:,.0f}  hand-offs/page {v[10] / pg:.1f}  " +
          "  ".join(f"{NAMES[k]} {100.0 * v[k] / max(tot, 1):.1f}%" for k in NAMES), flush=True)


if __name__ == "__main__":
    for plen in (16384, 32768):
        run(1, plen)
        run(4096, plen)
