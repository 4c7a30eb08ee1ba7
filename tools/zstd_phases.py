"""Diagnostic: where zstd decode pass 1 (zstd_entropy_kernel) spends its cycles (profile build).

    python -c "from tyche_amd import _build; _build.build(profile=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_prof.so PLEN=32768 PAGES=65536 python tools/zstd_phases.py

Per-page cycle stamps of wave 0 (clock64, SPROF_MARK in zstd_decode.hip): slot 1 = the whole
pass-1 page, 7 = Huffman tables (HUF_readStats + the decoding table), 2 = the rest of the
literals sections (the streams), 3 = sequence headers and FSE tables; 0 = pages.  Shares only: the stamps serialize the kernel a little.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402


def main():
    lib = _lib.load()
    prof = lib.tyche_debug_zstd_decode_profile
    prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    n = int(os.environ.get("PAGES", "65536"))
    plen = int(os.environ.get("PLEN", "32768"))
    pages = codec.pagegen(n, plen)
    comp, clen = codec.compress_pages(pages, compressor_id=3)
    torch.cuda.synchronize()
    mx = int(clen.max())
    buf = (ctypes.c_ulonglong * 16)()
    prof(buf, 1)
    out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=3, max_comp_len=mx)
    torch.cuda.synchronize()
    assert bool((rv == plen).all())
    prof(buf, 0)
    v = list(buf)
    pg = max(v[0], 1)
    total = v[1] / pg
    res = {"pages": n, "page_len": plen, "pass1_cycles_per_page": round(total),
           "huf_table_share": round(v[7] / pg / total, 3) if total else None,
           "literals_share": round(v[2] / pg / total, 3) if total else None,
           "seq_tables_share": round(v[3] / pg / total, 3) if total else None}
    res["rest_share"] = round(1 - (res["huf_table_share"] or 0) - (res["literals_share"] or 0) -
                              (res["seq_tables_share"] or 0), 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
