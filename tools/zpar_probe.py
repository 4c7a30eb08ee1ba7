"""Diagnostic for the lane-parallel zlib inflate: which bench pages the parallel path hands to
the serial decoder (TYCHE_ZLIB_PAR=2 reports them as INT32_MIN + 1), and per-batch kernel times
of both kernels for small batches (the restore path's sizes)."""
import os
import sys
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

dev = torch.device("cuda:0")
FALLBACK = -2**31 + 1
for plen in (16384, 32768):
    pages = codec.pagegen(4096, plen, dist=0, device=dev)
    comp, clen = codec.compress_pages(pages, compressor_id=2)
    host = [zlib.compress(pages[i].cpu().numpy().tobytes(), 1) for i in range(512)]
    torch.cuda.synchronize()
    mx = int(clen.max())
    for mode in ("2", "1", "0"):
        os.environ["TYCHE_ZLIB_PAR"] = mode
        out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=2, max_comp_len=mx)
        torch.cuda.synchronize()
        r = rv.cpu().numpy()
        line = {"plen": plen, "mode": mode, "device_streams": len(r), "ok": int((r == plen).sum()),
                "fallback": int((r == FALLBACK).sum())}
        if mode == "2":
            line["fallback_idx"] = [int(i) for i in np.nonzero(r == FALLBACK)[0][:12]]
            bad = np.nonzero(r != plen)[0]
            line["first_types"] = [int(comp[i, 2].item() & 7) for i in bad[:12]]
        # small-batch kernel times
        ts = {}
        for nb in (1, 8, 64, 512):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for rep in range(5):
                e0.record()
                codec.decompress_pages(comp[:nb], clen[:nb], plen, compressor_id=2, max_comp_len=mx)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1))
            ts[nb] = round(best * 1000, 1)
        line["batch_us"] = ts
        print(line, flush=True)
    os.environ["TYCHE_ZLIB_PAR"] = "2"
    L = max(len(h) for h in host)
    slots = np.zeros((len(host), (L + 127) // 128 * 128), np.uint8)
    for i, h in enumerate(host):
        slots[i, :len(h)] = np.frombuffer(h, np.uint8)
    out, rv = codec.decompress_pages(torch.from_numpy(slots).to(dev),
                                     torch.tensor([len(h) for h in host], dtype=torch.int32, device=dev), plen,
                                     compressor_id=2, max_comp_len=L)
    torch.cuda.synchronize()
    r = rv.cpu().numpy()
    print({"plen": plen, "host_zlib1_streams": len(r), "ok": int((r == plen).sum()), "fallback": int((r == FALLBACK).sum())},
          flush=True)
