"""Times the zlib inflate kernel on bench-distribution pages.

8192 distinct pages are compressed on the host with zlib level 1 (the
reference's level, src/options.c:68) and tiled over N slots; the kernel time is
taken with HIP events on the launch stream.  Prints ms per launch, GiB/s of
output and the implied ms per 1M pages.
"""
import os
import sys
import time
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tyche_amd import codec  # noqa: E402

n = int(os.environ.get("PAGES", "262144"))
plen = int(os.environ.get("PLEN", "16384"))
uniq = int(os.environ.get("UNIQ", "8192"))
level = int(os.environ.get("LEVEL", "1"))
dev = torch.device("cuda:0")
pages = codec.pagegen(uniq, plen, dist=int(os.environ.get("DIST", "0")), device=dev).cpu().numpy()
t0 = time.time()
comps = [zlib.compress(pages[i].tobytes(), level) for i in range(uniq)]
host_s = time.time() - t0
slot = (max(len(c) for c in comps) + 127) // 128 * 128
u = np.zeros((uniq, slot), np.uint8)
ul = np.zeros(uniq, np.int32)
for i, c in enumerate(comps):
    u[i, :len(c)] = np.frombuffer(c, np.uint8)
    ul[i] = len(c)
reps = (n + uniq - 1) // uniq
slots = torch.from_numpy(u).to(dev).repeat(reps, 1)[:n].contiguous()
clen = torch.from_numpy(ul).to(dev).repeat(reps)[:n].contiguous()
out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
rv = torch.empty((n,), dtype=torch.int32, device=dev)
codec.decompress_pages(slots, clen, plen, compressor_id=2, out=out, rv=rv)
torch.cuda.synchronize()
ok = bool((rv == plen).all()) and torch.equal(out[:uniq].cpu(), torch.from_numpy(pages[: min(uniq, n)]))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ts = []
for _ in range(3):
    ev[0].record()
    codec.decompress_pages(slots, clen, plen, compressor_id=2, out=out, rv=rv)
    ev[1].record()
    torch.cuda.synchronize()
    ts.append(ev[0].elapsed_time(ev[1]))
ms = min(ts)
ratio = plen * uniq / float(ul.sum())
print(f"zlib inflate: {n} x {plen} B  ratio {ratio:.3f}  {ms:.2f} ms  {n * plen / ms / 1e6 / 1.073741824:.1f} GiB/s  "
      f"({ms * (1 << 20) / n:.1f} ms per 1M pages)  correct={ok}  host zlib-{level} compress {uniq / host_s:.0f} pages/s")
