"""Diagnostic: LZ4 compress and decompress of 1M resident 16 KiB pages run back to back on one
stream, or at the same time on two streams with their residency capped so that both fit a CU's
LDS together (TYCHE_LZ4_ENC_PAGES_PER_CU encoder pages per CU, TYCHE_LZ4_LC_WAVES decoder waves
per CU: e.g. 4 x 29.9 KiB + 2 x 17.1 KiB < 160 KiB).  The encoder is bound by its CU's LDS, the
decoder by the memory side (profiles/r06_pmc_lz4_*.json), so co-resident waves may use units the
other leaves idle.  Decompress reads a compressed copy made before timing (as the bench's pipelined
step does: step k decodes what step k-1 encoded).  Prints ms per compress+decompress pair.

    PAIRS=4,2:4,8:5,8 python tools/time_corun.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

n = int(os.environ.get("PAGES", "1048576"))
plen = 16384
dev = torch.device("cuda:0")
pages = codec.pagegen(n, plen, device=dev)
comp0, clen0 = codec.compress_pages(pages)
comp1, clen1 = codec.compress_pages(pages)
torch.cuda.synchronize()
mx = int(clen0.max())
out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
rv = torch.empty((n,), dtype=torch.int32, device=dev)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def seq():
    codec.compress_pages(pages, out=comp1, out_len=clen1)
    codec.decompress_pages(comp0, clen0, plen, out=out, rv=rv, max_comp_len=mx)


def corun(dec_first):
    cur = torch.cuda.current_stream(dev)
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    order = [1, 0] if dec_first else [0, 1]
    for o in order:
        if o == 0:
            with torch.cuda.stream(sa):
                codec.compress_pages(pages, out=comp1, out_len=clen1)
        else:
            with torch.cuda.stream(sb):
                codec.decompress_pages(comp0, clen0, plen, out=out, rv=rv, max_comp_len=mx)
    cur.wait_stream(sa)
    cur.wait_stream(sb)


def timeit(fn, reps=4):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best


def check():
    torch.cuda.synchronize()
    ok = bool((rv == plen).all()) and torch.equal(out, pages) and torch.equal(clen0, clen1)
    assert ok, "round trip failed"


_lib.set_knob("LZ4_ENC_PAGES_PER_CU", 0)
_lib.set_knob("LZ4_LC_WAVES", 8)
t = timeit(seq)
check()
print(f"sequential (5 pages, 8 waves per CU): {t:7.2f} ms per pair  {2 * n * plen / t / 1e6 / 1.073741824:6.1f} GiB/s",
      flush=True)
for pair in os.environ.get("PAIRS", "4,2:4,8:3,4:5,8").split(":"):
    pe, wd = (int(x) for x in pair.split(","))
    _lib.set_knob("LZ4_ENC_PAGES_PER_CU", pe)
    _lib.set_knob("LZ4_LC_WAVES", wd)
    for dec_first in (True, False):
        out.zero_()
        t = timeit(lambda: corun(dec_first))
        check()
        print(f"corun enc {pe} pages/CU, dec {wd} waves/CU, {'decoder' if dec_first else 'encoder'} launched first: "
              f"{t:7.2f} ms per pair  {2 * n * plen / t / 1e6 / 1.073741824:6.1f} GiB/s", flush=True)
    # each alone at that residency
    _lib.set_knob("LZ4_LC_WAVES", wd)
    te = timeit(lambda: codec.compress_pages(pages, out=comp1, out_len=clen1))
    td = timeit(lambda: codec.decompress_pages(comp0, clen0, plen, out=out, rv=rv, max_comp_len=mx))
    print(f"   alone: encode {te:7.2f} ms, decode {td:7.2f} ms", flush=True)
