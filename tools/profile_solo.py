"""Diagnostic: per-phase cycles of the single-page LZ4 decoder (profile build).

    python -c "from tyche_amd import _build; _build.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so python tools/profile_solo.py
Wall cycles (clock64) per page and phase, stamped by lane 0 of each of the 16 waves (sums / 16).
Never quote its run time.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

NAMES = {1: "stage_in", 2: "next_positions", 3: "doubling", 4: "token_list", 5: "decode+checks+records",
         10: "cover_scan", 6: "cells", 7: "jump_rounds", 8: "pack_store"}


def main():
    lib = _lib.load()
    prof = lib.tyche_debug_decode_profile
    prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    plen = int(os.environ.get("PLEN", "16384"))
    for n in (1, 64, 2048):
        pages = codec.pagegen(n, plen, dist=int(os.environ.get("DIST", "0")))
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
        pg = max(v[9] / 16, 1)
        parts = "  ".join(f"{name} {v[k] / 16 / pg:.0f}" for k, name in NAMES.items())
        print(f"batch {n} x {plen}: {parts}  doubling_levels {v[11] / 16 / pg:.1f}  jump_rounds {v[12] / 16 / pg:.1f}"
              f"  pages {pg:.0f}", flush=True)


if __name__ == "__main__":
    main()
