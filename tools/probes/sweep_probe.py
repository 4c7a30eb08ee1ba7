"""Diagnostic: the sweep side of the C5 cycle -- one compressor-pool call (250 victims of 8/16/32 KiB,
tyche_compress_host LZ4) timed alone and from T threads at once, with the engine's host-stage clocks.

    python tools/probes/sweep_probe.py [threads=16] [calls_per_thread=20]
"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tyche_amd import _lib, codec  # noqa: E402


def batch(seed, n=250):
    rng = np.random.default_rng(seed)
    sizes = rng.choice([8192, 16384, 32768], n)
    pool = {s: codec.pagegen(n, s, seed=seed).cpu().numpy() for s in (8192, 16384, 32768)}
    pages = [pool[int(s)][i].copy() for i, s in enumerate(sizes)]
    caps = [codec.compress_bound(int(s)) for s in sizes]
    outs = [np.zeros(c, dtype=np.uint8) for c in caps]
    return pages, outs, caps


def main():
    nthr = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = _lib.load()
    cid = _lib.COMPRESSOR_IDS["lz4"]
    vp = ctypes.c_void_p
    batches = [batch(t + 1) for t in range(nthr)]
    args = []
    for pages, outs, caps in batches:
        n = len(pages)
        args.append(((vp * n)(*[p.ctypes.data for p in pages]), (ctypes.c_uint32 * n)(*[len(p) for p in pages]),
                     (vp * n)(*[o.ctypes.data for o in outs]), (ctypes.c_uint32 * n)(*caps), np.zeros(n, dtype=np.int32),
                     sum(len(p) for p in pages)))

    def call(t):
        s, sl, d, dc, res, _ = args[t]
        rc = lib.tyche_compress_host(cid, 1, len(res), s, sl, d, dc, res.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        assert rc == 0 and (res > 0).all()

    for _ in range(5):
        call(0)
    prof = (ctypes.c_uint64 * 8)()
    lib.tyche_host_profile(prof, 8)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        call(0)
        ts.append(time.perf_counter() - t0)
    lib.tyche_host_profile(prof, 8)
    raw = args[0][5]
    print(json.dumps({"threads": 1, "pages": 250, "raw_mib": round(raw / 2**20, 2), "ms_p50": round(np.median(ts) * 1e3, 2),
                      "gib_s": round(raw / np.median(ts) / 2**30, 3),
                      "per_call_ms": {k: round(prof[i] / calls / 1e6, 2) for i, k in
                                      enumerate(["stream_wait", "scatter", "gather", "enqueue"])}}), flush=True)

    def worker(t):
        for _ in range(calls):
            call(t)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nthr)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    tot = sum(a[5] for a in args) * calls
    print(json.dumps({"threads": nthr, "calls": nthr * calls, "s": round(dt, 3), "gib_s": round(tot / dt / 2**30, 3)}), flush=True)


if __name__ == "__main__":
    main()
