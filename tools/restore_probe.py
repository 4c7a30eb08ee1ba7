"""Diagnostic: where a single-page host restore's time goes (tyche_decompress_host, 1 page).

    python tools/restore_probe.py [codec=lz4] [page_len=16384] [reps=300]

For each setting of the zero-copy path (TYCHE_ZERO_COPY_BYTES default / 0) prints p50 / p90 us per call and
the engine's host-stage clocks per call (tyche_host_profile: stream wait = launch + kernel + completion
wake-up, gather, scatter, enqueue), next to the floor of an empty torch kernel launch + synchronize.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import _lib, codec  # noqa: E402


def main():
    cname = sys.argv[1] if len(sys.argv) > 1 else "lz4"
    plen = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    cid = _lib.COMPRESSOR_IDS[cname]
    lib = _lib.load()
    page = codec.pagegen(1, plen).cpu().numpy()[0].copy()
    cap = codec.compress_bound(plen)
    comp = np.zeros(cap, dtype=np.uint8)
    out = np.zeros(plen, dtype=np.uint8)
    res = np.zeros(1, dtype=np.int32)
    vp = ctypes.c_void_p * 1
    u32 = ctypes.c_uint32 * 1
    i32p = ctypes.POINTER(ctypes.c_int32)
    _lib.check(lib.tyche_compress_host(cid, 1, 1, vp(page.ctypes.data), u32(plen), vp(comp.ctypes.data), u32(cap),
                                       res.ctypes.data_as(i32p)), "compress")
    clen = int(res[0])
    # floor: an empty device op and a synchronize
    x = torch.zeros(1, device="cuda:0")
    for _ in range(50):
        x.add_(1)
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(json.dumps({"empty_kernel_sync_us_p50": round(float(np.median(ts)) * 1e6, 1)}), flush=True)
    for zc in (None, 0):
        if zc is None:
            _lib.clear_knob("ZERO_COPY_BYTES")
        else:
            _lib.set_knob("ZERO_COPY_BYTES", zc)
        # the call's arguments are built once: the timed region is the Buffer-API call, not the
        # construction of ctypes objects (numpy's .ctypes.data_as alone costs microseconds)
        args = (cid, 1, vp(comp.ctypes.data), u32(clen), vp(out.ctypes.data), u32(plen), res.ctypes.data_as(i32p))
        for _ in range(30):
            lib.tyche_decompress_host(*args)
        prof = (ctypes.c_uint64 * 8)()
        lib.tyche_host_profile(prof, 8)
        ts = []
        call = lib.tyche_decompress_host
        for _ in range(reps):
            t0 = time.perf_counter()
            rc = call(*args)
            ts.append(time.perf_counter() - t0)
            assert rc == 0 and res[0] == plen
        lib.tyche_host_profile(prof, 8)
        assert np.array_equal(out, page)
        ts = np.array(ts) * 1e6
        print(json.dumps({"codec": cname, "page_len": plen, "zero_copy": zc is None,
                          "us_p50": round(float(np.median(ts)), 1), "us_p90": round(float(np.percentile(ts, 90)), 1),
                          "per_call_us": {"stream_wait": round(prof[0] / reps / 1e3, 1),
                                          "scatter": round(prof[1] / reps / 1e3, 1),
                                          "gather": round(prof[2] / reps / 1e3, 1),
                                          "enqueue": round(prof[3] / reps / 1e3, 1)}}), flush=True)
    _lib.clear_knob("ZERO_COPY_BYTES")


if __name__ == "__main__":
    main()
