"""Diagnostic: per-stage cycle shares of the chunked lane-per-page LZ4 decoder (profile build).

    python -c "from tyche_amd import _build; _build.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so TYCHE_LZ4_LC=1 python tools/lc_profile.py
Shares only (the stamps serialize the kernel a little); never quote its run time.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

NAMES = {1: "parse_slots_0_1", 2: "store_drain_wait", 3: "parse_slots_2up+far_issue", 4: "general_slot",
         5: "window_issue", 6: "copy(far_wait)", 7: "window_wait+store", 8: "flush", 10: "tails+page_switch",
         9: "loop_top"}


def main():
    lib = _lib.load()
    prof = lib.tyche_debug_lc_profile
    prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    n = int(os.environ.get("PAGES", "262144"))
    plen = int(os.environ.get("PLEN", "16384"))
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
    tot = sum(v[k] for k in NAMES)
    chunks = max(v[0], 1)
    print(f"pages {n}  wave-chunks {v[0]} ({v[0] * 64 / n:.0f} per page-lane)  general slot taken in "
          f"{100.0 * v[12] / chunks:.1f} % of chunks  pieces flushed per chunk {v[13] / chunks:.1f}  page ends per chunk "
          f"{v[14] / chunks:.2f}")
    for k, name in NAMES.items():
        print(f"  {name:20s} {100.0 * v[k] / max(tot, 1):5.1f} %   {v[k] / chunks:8.0f} cycles per wave-chunk")


if __name__ == "__main__":
    main()
