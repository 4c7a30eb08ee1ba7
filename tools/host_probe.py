"""Diagnostic: where the host (PCIe-inclusive) path's time goes.

    python tools/host_probe.py [pages] [chunk_mb,...]

Prints JSON lines: the raw pinned H2D / D2H / bidirectional link rates (bench.pcie_probe),
then tyche_compress_host / tyche_decompress_host over `pages` malloc'd 16 KiB pages for each
HOST_CHUNK_MB setting (tyche_set_knob, read per call), best of 3 each; with AB_KNOB / AB_VALUES
also an interleaved A/B of one knob.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tyche_amd import _lib, codec  # noqa: E402

GIB = float(1 << 30)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    chunks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64, 32, 16]
    dev = torch.device("cuda:0")
    lib = _lib.load()
    plen = 16384
    pages = codec.pagegen(n, plen, device=dev)
    host = pages.cpu().numpy()
    print(json.dumps({"link": bench.pcie_probe(dev, n * plen)}), flush=True)
    cap = codec.compress_bound(plen)
    comp = np.zeros((n, cap), dtype=np.uint8)
    out = np.zeros_like(host)
    comp.fill(1)
    out.fill(1)   # touched: no first-write page faults in the timed calls
    res = np.zeros(n, dtype=np.int32)
    rv = np.zeros(n, dtype=np.int32)
    vp = ctypes.c_void_p * n
    src_p = vp(*[host.ctypes.data + i * plen for i in range(n)])
    comp_p = vp(*[comp.ctypes.data + i * cap for i in range(n)])
    out_p = vp(*[out.ctypes.data + i * plen for i in range(n)])
    u32 = ctypes.c_uint32 * n
    slen = u32(*([plen] * n))
    ccap = u32(*([cap] * n))
    i32p = ctypes.POINTER(ctypes.c_int32)
    def stages():
        prof = (ctypes.c_uint64 * 8)()
        lib.tyche_host_profile(prof, 8)
        return {"stream_wait_ms": prof[0] / 3e6, "scatter_ms": prof[1] / 3e6, "gather_ms": prof[2] / 3e6,
                "enqueue_ms": prof[3] / 3e6, "gather_gib": prof[4] / 3 / GIB, "scatter_gib": prof[5] / 3 / GIB,
                "chunks": prof[6] // 3}

    for mb in chunks:
        _lib.set_knob("HOST_CHUNK_MB", mb)
        nb = n * plen
        stages()
        bc = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            _lib.check(lib.tyche_compress_host(1, 1, n, src_p, slen, comp_p, ccap, res.ctypes.data_as(i32p)), "c")
            bc = min(bc, time.perf_counter() - t0)
        sc = stages()
        clen = u32(*[int(x) for x in res])
        bd = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            _lib.check(lib.tyche_decompress_host(1, n, comp_p, clen, out_p, slen, rv.ctypes.data_as(i32p)), "d")
            bd = min(bd, time.perf_counter() - t0)
        sd = stages()
        assert (rv == plen).all() and np.array_equal(out, host)
        print(json.dumps({"pages": n, "chunk_mb": mb, "compress_gib_s": round(nb / bc / GIB, 2),
                          "decompress_gib_s": round(nb / bd / GIB, 2),
                          "combined_gib_s": round(nb / (bc + bd) / GIB, 2),
                          "compress_ms": round(bc * 1e3, 2), "decompress_ms": round(bd * 1e3, 2),
                          "compress_stages_per_call": sc, "decompress_stages_per_call": sd}), flush=True)
    _lib.clear_knob("HOST_CHUNK_MB")
    # A/B of one knob in this process (AB_KNOB=name AB_VALUES=v1,v2): the values interleaved 5 times,
    # best call of each -- box-to-box variance of the host copies is larger than most differences
    ab = os.environ.get("AB_KNOB")
    if ab:
        vals = [int(v) for v in os.environ.get("AB_VALUES", "0,1").split(",")]
        best = {v: [float("inf"), float("inf")] for v in vals}
        for _ in range(5):
            for v in vals:
                _lib.set_knob(ab, v)
                t0 = time.perf_counter()
                _lib.check(lib.tyche_compress_host(1, 1, n, src_p, slen, comp_p, ccap, res.ctypes.data_as(i32p)), "c")
                best[v][0] = min(best[v][0], time.perf_counter() - t0)
                clen = u32(*[int(x) for x in res])
                t0 = time.perf_counter()
                _lib.check(lib.tyche_decompress_host(1, n, comp_p, clen, out_p, slen, rv.ctypes.data_as(i32p)), "d")
                best[v][1] = min(best[v][1], time.perf_counter() - t0)
        _lib.clear_knob(ab)
        nb = n * plen
        print(json.dumps({"ab_knob": ab, "pages": n, "best_of": 5,
                          "results": {str(v): {"compress_gib_s": round(nb / c / GIB, 2), "decompress_gib_s": round(nb / d / GIB, 2),
                                               "combined_gib_s": round(nb / (c + d) / GIB, 2)} for v, (c, d) in best.items()}}),
              flush=True)
    # host memcpy rate of the copy pool's work alone (numpy, one thread): scatter-sized copies
    a = np.ones(256 << 20, dtype=np.uint8)
    b = np.empty_like(a)
    t0 = time.perf_counter()
    for _ in range(4):
        np.copyto(b, a)
    print(json.dumps({"host_memcpy_1thread_gib_s": round(4 * a.size / (time.perf_counter() - t0) / GIB, 2)}))


if __name__ == "__main__":
    main()
