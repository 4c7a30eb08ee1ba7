"""Diagnostic: phase shares of the zstd encode and decode kernels (profile build).

    python -c "import tyche_amd._build as b; b.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so python tools/zstd_prof.py
Slot 1 is the whole page (encode: parse + blocks; decode: decode_frame); the others are
parts of it.  Cycles are clock64() deltas of lane 0 summed over pages."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

ENC = {2: "block sizes", 3: "literals (huf)", 4: "repeats+tables", 5: "FSE chain"}
DEC = {2: "literals", 3: "seq tables", 4: "FSE decode", 5: "exec", 6: "last literals"}


def show(tag, v, names):
    pg = max(v[0], 1)
    tot = v[1]
    print(f"{tag}: pages {v[0]}  cycles/page {tot / pg:,.0f}  seq/page {v[9] / pg:.0f}  " +
          "  ".join(f"{names[k]} {100.0 * v[k] / max(tot, 1):.1f}%" for k in names) +
          f"  rest {100.0 * (tot - sum(v[k] for k in names)) / max(tot, 1):.1f}%", flush=True)


def main():
    lib = _lib.load()
    fns = {}
    for k in ("encode", "decode"):
        f = getattr(lib, f"tyche_debug_zstd_{k}_profile")
        f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        fns[k] = f
    for plen, n in ((32768, 1), (32768, 16384), (16384, 16384)):
        pages = codec.pagegen(max(n, 64), plen, dist=0)[:n].contiguous()
        buf = (ctypes.c_ulonglong * 16)()
        fns["encode"](buf, 1)
        comp, clen = codec.compress_pages(pages, compressor_id=3)
        torch.cuda.synchronize()
        fns["encode"](buf, 0)
        show(f"encode n={n} plen={plen}", list(buf), ENC)
        fns["decode"](buf, 1)
        out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=3, max_comp_len=int(clen.max()))
        torch.cuda.synchronize()
        assert bool((rv == plen).all()) and torch.equal(out, pages)
        fns["decode"](buf, 0)
        show(f"decode n={n} plen={plen}", list(buf), DEC)


if __name__ == "__main__":
    main()
