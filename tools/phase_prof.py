"""Per-phase cycle attribution of the LZ4 encoder's parse (profiling build only).

    python /tmp/mkvar.py ph=-DTYCHE_PHASES   # or any build with -DTYCHE_PHASES
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_ph.so PAGES=262144 python tools/phase_prof.py
Phases: 0 block scan (hash, lookup, insert, verify, probes, ballot), 1 greedy walk
(without 5), 2 record append, 3 sink (sequence encoding and byte emission),
4 loop exit, 5 whole-wave extension of probe-capped matches.  Prints wave cycles per page for each.
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec, _lib  # noqa: E402

n = int(os.environ.get("PAGES", "262144"))
plen = int(os.environ.get("PLEN", "16384"))
pages = codec.pagegen(n, plen)
comp, clen = codec.compress_pages(pages)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * 16)()
assert lib.tyche_phase_read(buf) == 0, "tyche_phase_read failed"
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
codec.compress_pages(pages, out=comp, out_len=clen)
e1.record()
torch.cuda.synchronize()
assert lib.tyche_phase_read(buf) == 0, "tyche_phase_read failed"
npg = buf[7]
names = ["block scan", "greedy walk", "record append", "sink/emit", "exit", "wave extend"]
tot = sum(buf[i] for i in range(6))
for i, nm in enumerate(names):
    print(f"{nm:14s} {buf[i] / npg:10.0f} cycles/page  {100.0 * buf[i] / tot:5.1f} %")
print(f"extensions     {buf[6] / npg:10.1f} per page; blocks {buf[8] / npg:.1f}, with a match {buf[10] / npg:.1f}, matches {buf[9] / npg:.1f}")
print(f"parse total    {tot / npg:10.0f} cycles/page; kernel {e0.elapsed_time(e1):.2f} ms for {n} pages; pages seen {npg}")
if buf[15]:
    sub = ["fields + prefix sum", "ring writes", "long literal runs", "ring flush"]
    st = sum(buf[11 + i] for i in range(4))
    print(f"sink sub-phases (every 64th workgroup, {buf[15]} calls):")
    for i, nm in enumerate(sub):
        print(f"  {nm:20s} {buf[11 + i] / buf[15]:8.0f} cycles/call  {100.0 * buf[11 + i] / st:5.1f} %")

