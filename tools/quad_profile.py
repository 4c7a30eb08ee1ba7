"""Diagnostic: per-stage cycle shares of the quad-per-page LZ4 decoder (profile build).

    python -c "from tyche_amd import _build; _build.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so TYCHE_LZ4_QUAD=1 python tools/quad_profile.py
Shares only (the stamps serialize the kernel a little); never quote its run time.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

NAMES = {1: "stage1_parse", 2: "stage2_far_wait", 3: "stage3_copy", 4: "stage4_flush", 5: "stage5_slow_path",
         6: "stage5_page_switch", 7: "stage5_window_write"}


def main():
    lib = _lib.load()
    prof = lib.tyche_debug_quad_profile
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
    print(f"pages {n}  wave-chunks {v[0]}  per 16-page wave-chunk: parse iterations {v[8] / chunks:.1f}, "
          f"records {v[12] / n:.0f}/page ({v[12] / max(v[0], 1) / 16:.1f} per slot-chunk), far {v[13] / n:.0f}/page, "
          f"breakers {v[10] / n:.2f}/page, page ends {v[11] / n:.2f}/page")
    for k, name in NAMES.items():
        print(f"  {name:20s} {100.0 * v[k] / max(tot, 1):5.1f} %   {v[k] / chunks:8.0f} cycles per wave-chunk")


if __name__ == "__main__":
    main()
