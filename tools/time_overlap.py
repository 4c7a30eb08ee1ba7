"""Diagnostic: compress+decompress of N resident pages, sequential vs pipelined in K
chunks on two HIP streams (chunk k's decode overlaps chunk k+1's encode, as sweep
and restore overlap in tyche).  Prints ms per pass and GiB/s; checks the round trip.

    PAGES=1048576 KS=2,4,8 python tools/time_overlap.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

n = int(os.environ.get("PAGES", "1048576"))
plen = int(os.environ.get("PLEN", "16384"))
ks = [int(k) for k in os.environ.get("KS", "2,4,8").split(",")]
dev = torch.device("cuda:0")
pages = codec.pagegen(n, plen, device=dev)
comp = torch.empty((n, codec.slot_size(plen)), dtype=torch.uint8, device=dev)
clen = torch.empty((n,), dtype=torch.int32, device=dev)
out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
rv = torch.empty((n,), dtype=torch.int32, device=dev)
codec.compress_pages(pages, out=comp, out_len=clen)
torch.cuda.synchronize()
mx = int(clen.max())


def seq():
    codec.compress_pages(pages, out=comp, out_len=clen)
    codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=mx)


sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def pipe(k):
    step = (n + k - 1) // k
    cur = torch.cuda.current_stream(dev)
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    for c in range(k):
        a, b = c * step, min(n, (c + 1) * step)
        with torch.cuda.stream(sa):
            codec.compress_pages(pages[a:b], out=comp[a:b], out_len=clen[a:b])
            ev = torch.cuda.Event()
            ev.record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(ev)
            codec.decompress_pages(comp[a:b], clen[a:b], plen, out=out[a:b], rv=rv[a:b], max_comp_len=mx)
    cur.wait_stream(sa)
    cur.wait_stream(sb)


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    rv.zero_()
    out.zero_()
    fn()
    torch.cuda.synchronize()
    ok = bool((rv == plen).all()) and torch.equal(out, pages)
    return best * 1e3, ok


gib = n * plen / 2**30
ms, ok = timeit(seq)
print(f"sequential: {ms:8.2f} ms  {gib / ms * 1e3:7.1f} GiB/s  ok={ok}", flush=True)
for k in ks:
    ms, ok = timeit(lambda: pipe(k))
    print(f"pipelined K={k}: {ms:8.2f} ms  {gib / ms * 1e3:7.1f} GiB/s  ok={ok}", flush=True)
