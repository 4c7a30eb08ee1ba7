"""Diagnostic: where the large-batch LZ4 decoder's time goes, by making its memory traffic cache-resident.

Three decodes of the same number of pages through the ragged batch form (per-page offsets):
  distinct  every page has its own stream and its own output row (the bench layout);
  stream    every page's stream aliases one of U compressed pages (the stream lines stay in L2/MALL),
            outputs distinct;
  both      streams alias U pages and outputs alias U rows as well (all lanes decoding the same page
            write the same bytes to the same place, so far-match reads of that row hit L2 too).
The parse, the records and the copies are the same work in all three; the differences are the cost
of the stream fetches and of the output stores / far reads missing the caches.

    PAGES=262144 UNIQUE=2048 python tools/lc_alias.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402


def main():
    n = int(os.environ.get("PAGES", "262144"))
    u = int(os.environ.get("UNIQUE", "2048"))
    plen = int(os.environ.get("PLEN", "16384"))
    dev = torch.device("cuda:0")
    pages = codec.pagegen(n, plen, dist=int(os.environ.get("DIST", "0")), device=dev)
    comp, clen = codec.compress_pages(pages)
    torch.cuda.synchronize()
    slot = comp.shape[1]
    mx = int(clen.max())
    flat = comp.reshape(-1)
    idx = torch.arange(n, device=dev, dtype=torch.int64)
    alias = idx % u
    caps = torch.full((n,), plen, dtype=torch.int32, device=dev)
    out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
    rv = torch.empty((n,), dtype=torch.int32, device=dev)

    def run(src_idx, dst_idx):
        offs = (src_idx * slot).contiguous()
        lens = clen[src_idx].contiguous()
        oofs = (dst_idx * plen).contiguous()
        args = (flat, offs, lens, caps, out.reshape(-1), oofs, rv, mx, plen)
        codec.decompress_ragged(*args)
        torch.cuda.synchronize()
        ok = bool((rv == plen).all())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            codec.decompress_ragged(*args)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best * (1 << 20) / n, ok

    res = {"pages": n, "unique": u, "page_len": plen}
    for name, s, d in (("distinct", idx, idx), ("stream", alias, idx), ("both", alias, alias)):
        ms, ok = run(s, d)
        res[name + "_ms_per_1M"] = round(ms, 2)
        res[name + "_ok"] = ok
    print(json.dumps(res))


if __name__ == "__main__":
    main()
