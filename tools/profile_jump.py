"""Diagnostic: per-phase cycles of the LZ4 jump decoder (profile build).

    python -c "from tyche_amd import _build; _build.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so python tools/profile_jump.py
Wall cycles (clock64) per page and phase; workgroup-wide phases are stamped by the lane 0
of each of the 8 waves, so their sums are divided by 8.  Never quote its run time.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

WG = {0: "pages", 1: "stage_in", 5: "front_total", 6: "checks_fills+long_runs", 7: "scan_fill", 8: "jump_rounds", 12: "pack_store", 9: "rounds", 10: "long_runs"}
W0 = {2: "chain_walk", 3: "chain_bridge", 4: "walk_items"}


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
        if not os.environ.get("PROF_NOCHECK"):
            assert bool((rv == plen).all()) and torch.equal(out, pages)
        prof(buf, 0)
        v = list(buf)
        pg = max(v[0] / 8, 1)
        parts = {name: v[k] / 8 / pg for k, name in WG.items() if k not in (0,)}
        parts.update({name: v[k] / pg for k, name in W0.items()})
        print(f"batch {n} x {plen}: " + "  ".join(f"{k} {val:.0f}" for k, val in parts.items()), flush=True)


if __name__ == "__main__":
    main()
