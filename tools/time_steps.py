"""Diagnostic: per-step kernel times of the bench's C2 step (LZ4 compress then decompress of 1M
resident 16 KiB pages, the same buffers every step), one line per step, for each LZ4 decoder ring
size in RINGS (TYCHE_LZ4_LC_RING).  Shows whether single slow decode calls recur.

    RINGS=192,160 STEPS=10 python tools/time_steps.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

n = int(os.environ.get("PAGES", "1048576"))
plen = 16384
dev = torch.device("cuda:0")
pages = codec.pagegen(n, plen, device=dev)
comp = torch.empty((n, codec.slot_size(plen)), dtype=torch.uint8, device=dev)
clen = torch.empty((n,), dtype=torch.int32, device=dev)
out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
rv = torch.empty((n,), dtype=torch.int32, device=dev)
codec.compress_pages(pages, out=comp, out_len=clen)
torch.cuda.synchronize()
mx = int(clen.max())
# BETWEEN (per block, comma-separated): "knob" sets the ring knob, "check" runs the bench's
# round-trip check (torch kernels over out and pages; "chunked": in 1 GiB slices), "alloc" /
# "alloc_empty" a fresh 16 GiB tensor written once / never, "sleep" idles the host 50 ms, "none"
between = os.environ.get("BETWEEN", "knob").split(",")
rings = [int(x) for x in os.environ.get("RINGS", "192,160").split(",")]
for bi, ring in enumerate(rings):
    what = between[bi % len(between)]
    if what == "knob":
        _lib.set_knob("LZ4_LC_RING", ring)
    elif what == "check":
        assert bool((rv == plen).all()) and torch.equal(out, pages)
    elif what == "chunked":   # the same check in 1 GiB slices (one 1 GiB temporary, reused)
        step = (1 << 30) // plen
        ok = bool((rv == plen).all())
        for a in range(0, n, step):
            ok = ok and torch.equal(out[a:a + step], pages[a:a + step])
        assert ok
    elif what == "alloc":     # a fresh 16 GiB allocation, written once and freed back to torch's cache
        x = torch.empty((n, plen), dtype=torch.bool, device=dev)
        x.fill_(True)
        del x
    elif what == "alloc_empty":   # the same allocation, never written
        x = torch.empty((n, plen), dtype=torch.bool, device=dev)
        del x
    elif what == "sleep":
        import time
        time.sleep(0.05)
    print(json.dumps({"block": bi, "between": what}), flush=True)
    for k in range(int(os.environ.get("STEPS", "10"))):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        codec.compress_pages(pages, out=comp, out_len=clen)
        ev[1].record()
        codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=mx)
        ev[2].record()
        torch.cuda.synchronize()
        print(json.dumps({"ring": ring, "between": what, "step": k, "encode_ms": round(ev[0].elapsed_time(ev[1]), 3),
                          "decode_ms": round(ev[1].elapsed_time(ev[2]), 3)}), flush=True)
torch.cuda.synchronize()
assert bool((rv == plen).all()) and torch.equal(out, pages)
