"""Turns the two rocprofv3 PMC passes of tools/run_codec.py into HBM bytes per page.

    python tools/pmc_traffic.py <reads.csv> <WRITE_SIZE.csv> --pages 1048576 --page-len 16384 -o out.json

Reads: the `rdreq` pass of tools/gpu_traffic.sh (TCC_EA0_RDREQ_DRAM_32B_sum: the L2's
memory-side read requests in 32-byte units, a 128-byte request counted as 4), read bytes =
32 * that count.  Round 6's calibration (tools/probes/fetch_calib.hip,
profiles/r06_fetch_calib.json) shows every gfx950 read request is a 128-byte line --
coalesced 16/8/1-byte streams and scattered 16-byte loads alike (TCC_EA0_RDREQ_sum * 4 =
TCC_EA0_RDREQ_DRAM_32B_sum, TCC_BUBBLE_sum ~0) -- and that FETCH_SIZE counts each at 64
bytes: with a FETCH_SIZE pass instead, read bytes = 2 * FETCH_SIZE for every kernel.
(Rounds 2-5 took the lane LZ4 decoder's FETCH_SIZE at face value -- r02_fetch_calib.json
read a 16-byte random load's one request as 64 bytes -- and so reported half its reads.)
WRITE_SIZE is in KiB and taken as is.  Each kernel's figure is
its bytes per codec call divided by the pages of a call.  A call is one
dispatch, except where --calls says how many calls the kernel's dispatches
make up (the LZ4 decoder runs two size-class launches per call:
--calls lz4_decode=1 for tools/run_codec.py with REPS=1; the split zstd codec
runs 3-4 kernels per chunk of pages: --calls zstd_encode=2 --calls zstd_decode=1).
bench.py scales the per-page figure to its own launch for `roofline.traffic`.
"""
import argparse
import csv
import json
import os
import subprocess
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd._build import kernel_sources_digest  # noqa: E402

# codec call -> the kernel symbols its dispatches carry (the split zstd codec runs several
# kernels per chunk of pages and several chunks per call: give --calls for it)
KERNELS = {"lz4_encode": ("lz4_encode_",), "lz4_decode": ("lz4_decode_",),
           "zstd_encode": ("zstd_encode_kernel", "zstd_parse_split_kernel", "zstd_block_kernel", "zstd_fse_kernel",
                           "zstd_pack_kernel"),
           "zstd_decode": ("zstd_decode_kernel", "zstd_entropy_kernel", "zstd_seq_kernel", "zstd_exec_kernel",
                           "zstd_exec_lane_kernel", "zstd_seqexec_kernel", "zstd_lit_kernel"),
           "zlib_encode": ("zlib_deflate_kernel",), "zlib_decode": ("zlib_inflate_kernel",)}


RDREQ = "TCC_EA0_RDREQ_DRAM_32B_sum"


def per_dispatch(path, counter):
    """kernel -> list of per-dispatch values in KiB: read bytes for `reads` (RDREQ * 32 B, or
    2 * FETCH_SIZE), WRITE_SIZE as is."""
    acc = defaultdict(float)
    names = {}
    rows = list(csv.DictReader(open(path)))
    if counter == "reads":
        counter = RDREQ if any(r["Counter_Name"] == RDREQ for r in rows) else "FETCH_SIZE"
    for r in rows:
        if r["Counter_Name"] != counter:
            continue
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = defaultdict(list)
    for d, v in acc.items():
        v *= 32.0 / 1024.0 if counter == RDREQ else 2.0 if counter == "FETCH_SIZE" else 1.0
        for k, syms in KERNELS.items():
            if any(sym in names[d] for sym in syms):
                out[k].append(v)
    return out


def _head():
    try:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        return subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except (OSError, subprocess.SubprocessError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch", help="the rdreq (or FETCH_SIZE) pass")
    ap.add_argument("write")
    ap.add_argument("--pages", type=int, required=True)
    ap.add_argument("--page-len", type=int, default=16384)
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--calls", action="append", default=[], help="kernel=N: its dispatches make up N codec calls")
    a = ap.parse_args()
    calls = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.calls}
    f = per_dispatch(a.fetch, "reads")
    w = per_dispatch(a.write, "WRITE_SIZE")
    res = {"pages_per_call": a.pages, "page_len": a.page_len, "calls": calls,
           "formula": "(read bytes + WRITE_SIZE * 1024) / pages; read bytes = 32 * TCC_EA0_RDREQ_DRAM_32B_sum "
                      "(or 2 * 1024 * FETCH_SIZE: gfx950 read requests are 128-byte lines counted at 64 B, every "
                      "access pattern, profiles/r06_fetch_calib.json)",
           "bytes_per_page": {}, "read_bytes_per_page": {}, "write_bytes_per_page": {},
           # the kernel code these counters describe: bench.py reports `traffic` only while this
           # digest equals the digest of the sources it runs (a stale summary must not look current)
           "kernel_sources_sha16": kernel_sources_digest(), "commit": _head()}
    for k in KERNELS:
        if not f.get(k) or not w.get(k):
            continue
        nf, nw = calls.get(k, len(f[k])), calls.get(k, len(w[k]))
        rd = 1024 * sum(f[k]) / nf / a.pages
        wr = 1024 * sum(w[k]) / nw / a.pages
        res["read_bytes_per_page"][k] = round(rd, 1)
        res["write_bytes_per_page"][k] = round(wr, 1)
        res["bytes_per_page"][k] = round(rd + wr, 1)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
