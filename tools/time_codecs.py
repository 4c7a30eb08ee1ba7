"""Times every device codec on bench-distribution pages (HIP events on the launch stream).

For each (codec, page size): one device compress pass and one device decompress
pass over N resident pages (own frames), plus -- for zstd and zlib -- a decode
pass over frames made by the reference's own level-1 encoder (oracle/_ref,
UNIQ distinct pages tiled over N slots), which exercises the Huffman-literal /
dynamic-tree decode paths the device encoders do not emit.

    PAGES=262144 python tools/time_codecs.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

GIB = float(1 << 30)
n = int(os.environ.get("PAGES", "262144"))
uniq = int(os.environ.get("UNIQ", "4096"))
reps = int(os.environ.get("REPS", "3"))
dev = torch.device("cuda:0")
IDS = {"lz4": 1, "zlib": 2, "zstd": 3}


def timed(fn):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = float("inf")
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]))
    return best


def own(name, plen):
    cid = IDS[name]
    pages = codec.pagegen(n, plen, dist=0, device=dev)
    comp, clen = codec.compress_pages(pages, compressor_id=cid)
    torch.cuda.synchronize()
    mx = int(clen.max())
    out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=cid, max_comp_len=mx)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages), name
    c_ms = timed(lambda: codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen))
    d_ms = timed(lambda: codec.decompress_pages(comp, clen, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx))
    nbytes = n * plen
    cb = int(clen.to(torch.int64).sum())
    r = {"codec": name, "page_len": plen, "pages": n, "ratio": round(nbytes / cb, 3),
         "compress_ms": round(c_ms, 3), "decompress_ms": round(d_ms, 3),
         "compress_gib_s": round(nbytes / c_ms / 1e-3 / GIB, 2), "decompress_gib_s": round(nbytes / d_ms / 1e-3 / GIB, 2),
         "combined_gib_s": round(nbytes / (c_ms + d_ms) / 1e-3 / GIB, 2),
         "compress_hbm_frac": round((nbytes + cb) / c_ms / 1e-3 / 8e12, 4),
         "decompress_hbm_frac": round((nbytes + cb) / d_ms / 1e-3 / 8e12, 4)}
    del pages, comp, clen, out, rv
    torch.cuda.empty_cache()
    return r


def ref_frames(name, plen):
    from oracle import oracle as O
    if not O.have_ref():
        return None
    cid = IDS[name]
    host = codec.pagegen(uniq, plen, dist=0, device=dev).cpu().numpy()
    enc = O.ref_zstd_compress if name == "zstd" else O.ref_zlib_compress
    comps = [enc(host[i].tobytes(), 1) for i in range(uniq)]
    slot = (max(len(c) for c in comps) + 127) // 128 * 128
    u = np.zeros((uniq, slot), np.uint8)
    ul = np.zeros(uniq, np.int32)
    for i, c in enumerate(comps):
        u[i, :len(c)] = np.frombuffer(c, np.uint8)
        ul[i] = len(c)
    k = (n + uniq - 1) // uniq
    slots = torch.from_numpy(u).to(dev).repeat(k, 1)[:n].contiguous()
    clen = torch.from_numpy(ul).to(dev).repeat(k)[:n].contiguous()
    out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
    rv = torch.empty((n,), dtype=torch.int32, device=dev)
    mx = int(ul.max())
    codec.decompress_pages(slots, clen, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out[:uniq].cpu(), torch.from_numpy(host)), name
    d_ms = timed(lambda: codec.decompress_pages(slots, clen, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx))
    nbytes = n * plen
    return {"codec": name + " (reference level-1 frames)", "page_len": plen, "pages": n,
            "ratio": round(plen * uniq / float(ul.sum()), 3), "decompress_ms": round(d_ms, 3),
            "decompress_gib_s": round(nbytes / d_ms / 1e-3 / GIB, 2)}


if __name__ == "__main__":
    which = os.environ.get("CODECS", "lz4:16384,zstd:32768,zstd:16384,zlib:16384").split(",")
    for w in which:
        name, plen = w.split(":")
        print(json.dumps(own(name, int(plen))), flush=True)
        if name != "lz4" and os.environ.get("REF", "1") == "1":
            r = ref_frames(name, int(plen))
            if r:
                print(json.dumps(r), flush=True)
