"""Diagnostic: kernel time of the lane-parallel zlib inflate per page (one page per launch) over the
first N bench pages, to find pages the parallel path handles slowly; with a profile build
(TYCHE_CODEC_LIB=...prof.so) also the phase shares of the slowest page."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402

dev = torch.device("cuda:0")
N = int(os.environ.get("N", "64"))
for plen in (16384, 32768):
    pages = codec.pagegen(N, plen, dist=0, device=dev)
    comp, clen = codec.compress_pages(pages, compressor_id=2)
    torch.cuda.synchronize()
    mx = int(clen.max())
    times = []
    for i in range(N):
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            codec.decompress_pages(comp[i:i + 1], clen[i:i + 1], plen, compressor_id=2, max_comp_len=mx)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        times.append(best * 1000)
    order = sorted(range(N), key=lambda i: -times[i])
    print({"plen": plen, "median_us": round(sorted(times)[N // 2], 1),
           "slowest": [(i, round(times[i], 1), int(clen[i]), int(comp[i, 2].item()) & 7) for i in order[:6]]}, flush=True)
    lib = _lib.load()
    if hasattr(lib, "tyche_debug_zlib_profile"):
        prof = lib.tyche_debug_zlib_profile
        prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        for i in (order[0], order[N // 2]):
            buf = (ctypes.c_ulonglong * 16)()
            prof(buf, 1)
            codec.decompress_pages(comp[i:i + 1], clen[i:i + 1], plen, compressor_id=2, max_comp_len=mx)
            torch.cuda.synchronize()
            prof(buf, 0)
            v = list(buf)
            names = {1: "tables", 2: "walk", 3: "bridge", 4: "count", 5: "write", 6: "matches", 8: "adler"}
            tot = sum(v[k] for k in names)
            print("  page", i, "cycles", tot, "hand-offs", v[10], "rounds", v[11], "batches", v[12], "matches", v[13],
                  "scan/flush cycles", v[14], v[15], " ".join(f"{names[k]} {100 * v[k] / max(tot, 1):.0f}%" for k in names),
                  flush=True)
