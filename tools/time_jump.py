"""Diagnostic: LZ4 decode time of the small-batch decoders per batch size (single-page decoder, jump
decoder at 1,024 / 512 threads, wave decoder; MODES selects).

    python tools/time_jump.py            # prints one JSON line per (decoder, page_len, batch)
Each decoder runs in a child process (TYCHE_LZ4_JUMP_MAX is read once per process):
jump = every batch below the lane threshold on lz4_decode_jump_kernel, wave = none.
Times are HIP events around the decompress call on device-resident pages (median of reps).
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from tyche_amd import codec
mode = os.environ["MODE"]
for plen in (16384, 32768):
    big = codec.pagegen(16384, plen, dist=0)
    comp_all, clen_all = codec.compress_pages(big)
    torch.cuda.synchronize()
    for n in (1, 8, 64, 512, 4096, 16384):
        comp, clen, pages = comp_all[:n].contiguous(), clen_all[:n].contiguous(), big[:n]
        mx = int(clen.max())
        out, rv = codec.decompress_pages(comp, clen, plen, max_comp_len=mx)
        torch.cuda.synchronize()
        ok = bool((rv == plen).all()) and torch.equal(out, pages)
        ts = []
        reps = 20 if n < 4096 else 5
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=mx); e1.record()
            torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
        ts.sort()
        t = ts[len(ts) // 2]
        print(json.dumps({"decoder": mode, "page_len": plen, "batch": n, "us": round(t * 1000, 1),
                          "GiBps": round(n * plen / (t / 1000) / 2**30, 2), "correct": ok}), flush=True)
'''


ZCHILD = r'''
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from tyche_amd import codec
for plen in (16384, 32768):
    big = codec.pagegen(2048, plen, dist=0)
    comp_all, clen_all = codec.compress_pages(big, compressor_id=2)
    torch.cuda.synchronize()
    for n in (1, 8, 64, 512):
        comp, clen, pages = comp_all[:n].contiguous(), clen_all[:n].contiguous(), big[:n]
        mx = int(clen.max())
        for mode, jmax, wg in (("zlib-jump-wg", "1024", "1"), ("zlib-jump-wave", "1024", "0"), ("zlib-frontier", "0", "1")):
            os.environ["TYCHE_ZLIB_JUMP_MAX"] = jmax
            os.environ["TYCHE_ZLIB_JUMP_WG"] = wg
            out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=2, max_comp_len=mx)
            torch.cuda.synchronize()
            ok = bool((rv == plen).all()) and torch.equal(out, pages)
            ts = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); codec.decompress_pages(comp, clen, plen, compressor_id=2, out=out, rv=rv, max_comp_len=mx); e1.record()
                torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
            ts.sort()
            t = ts[len(ts) // 2]
            print(json.dumps({"decoder": mode, "page_len": plen, "batch": n, "us": round(t * 1000, 1),
                              "GiBps": round(n * plen / (t / 1000) / 2**30, 2), "correct": ok}), flush=True)
'''


def main():
    if os.environ.get("ZLIB", "1") != "0":
        r = subprocess.run([sys.executable, "-c", ZCHILD], capture_output=True, text=True, timeout=600)
        print(r.stdout.strip() or r.stderr.strip()[-1500:], flush=True)
    if os.environ.get("LZ4", "1") == "0":
        return
    modes = os.environ.get("MODES", "solo,jump,jump512,wave").split(",")
    table = {"solo": ("4096", "32767", "1"), "jump": ("0", "32767", "1"), "jump512": ("0", "32767", "0"),
             "wave": ("0", "0", "1")}
    for mode in modes:
        smax, jmax, wide = table[mode]
        env = dict(os.environ, MODE=mode, TYCHE_LZ4_SOLO_MAX=smax, TYCHE_LZ4_JUMP_MAX=jmax, TYCHE_LZ4_JUMP_WIDE=wide)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
        print(r.stdout.strip() or r.stderr.strip()[-1500:], flush=True)


if __name__ == "__main__":
    main()
