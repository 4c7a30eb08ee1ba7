"""Turns the two rocprofv3 PMC passes of tools/run_codec.py into HBM bytes per page.

    python tools/pmc_traffic.py profiles/r01_pmc_fetch_size.csv profiles/r01_pmc_write_size.csv \
        --pages 262144 --page-len 16384 -o profiles/r01_traffic.json

Correction: FETCH_SIZE and WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced 16-B/lane streaming read (MI355X_MICROARCH.md,
HBM section): the kernels that stage whole pages into LDS read that way, so
their read bytes are 2 * FETCH_SIZE.  The lane-per-page LZ4 decoder reads
scattered 16-byte pieces, one lane per page; for that pattern the calibration
probe (tools/probes/fetch_calib.hip, profiles/r02_fetch_calib.json) shows
FETCH_SIZE = 64 B per fabric read request = the bytes actually fetched, so its
read bytes are 1 * FETCH_SIZE.  Each kernel's figure is
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


# read-byte factor per FETCH_SIZE byte, by kernel symbol (see the module docstring)
SCATTERED = ("lz4_decode_ring_kernel", "lz4_decode_ringlb_kernel", "lz4_decode_lane_kernel", "lz4_decode_quad_kernel",
             "lz4_decode_lc_kernel",
             "zstd_seq_kernel",
             "zstd_fse_kernel", "zstd_exec_lane_kernel", "zstd_seqexec_kernel", "zstd_lit_kernel")


def per_dispatch(path, counter):
    """kernel -> list of per-dispatch values; FETCH_SIZE already scaled to read bytes (KiB)."""
    acc = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = defaultdict(list)
    for d, v in acc.items():
        if counter == "FETCH_SIZE":
            v *= 1.0 if any(sym in names[d] for sym in SCATTERED) else 2.0
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
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--pages", type=int, required=True)
    ap.add_argument("--page-len", type=int, default=16384)
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--calls", action="append", default=[], help="kernel=N: its dispatches make up N codec calls")
    a = ap.parse_args()
    calls = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.calls}
    f = per_dispatch(a.fetch, "FETCH_SIZE")
    w = per_dispatch(a.write, "WRITE_SIZE")
    res = {"pages_per_call": a.pages, "page_len": a.page_len, "calls": calls,
           "formula": "(c*FETCH_SIZE + WRITE_SIZE) * 1024 / pages; c = 2 for the page-staging kernels (gfx950 "
                      "half count of coalesced streaming reads), 1 for the scattered lane LZ4 decoder (calibrated, "
                      "tools/probes/fetch_calib.hip)",
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
