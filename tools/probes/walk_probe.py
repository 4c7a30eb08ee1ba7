"""Diagnostic: cycles per token of the one-wave serial LZ4 token walk (walk_probe.hip) on bench
pages of every distribution and on crafted 3-byte-sequence streams; checks the walked chain
against the token chain restated on the host (oracle's LZ4 stream walk).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probes/walk_probe.hip -o tools/probes/libwalk_probe.so
    python tools/probes/walk_probe.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tyche_amd import codec  # noqa: E402


def host_chain(s):
    """Token positions and output offsets along the chain (solo_next's rules)."""
    L = len(s)
    p, d, out = 0, 0, []
    while p < L:
        t = s[p]
        q, lit = p + 1, t >> 4
        if lit == 15:
            b = s[q] if q < L else 0
            q += 1
            lit += b
            while q < L - 15 and b == 255:
                b = s[q]
                q += 1
                lit += b
        out.append((p, d))
        if q + lit > L - 8:
            break
        q2, ml = q + lit + 2, t & 15
        bad = False
        if ml == 15:
            while True:
                b = s[q2]
                q2 += 1
                if q2 > L - 5:
                    bad = True
                    break
                ml += b
                if b != 255:
                    break
        if bad:
            break
        d += lit + ml + 4
        p = q2
    return out


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools/probes/libwalk_probe.so"))
    dev = torch.device("cuda:0")
    rows = []
    for dist in range(6):
        pages = codec.pagegen(8, 16384, dist=dist, first=dist * 100, device=dev)
        comp, clen = codec.compress_pages(pages)
        torch.cuda.synchronize()
        for i in range(8):
            L = int(clen[i])
            if L >= 8192:
                continue
            src = comp[i, :L].contiguous()
            lst = torch.zeros(8192, dtype=torch.int32, device=dev)
            cnt = torch.zeros(1, dtype=torch.int32, device=dev)
            cyc = torch.zeros(1, dtype=torch.int64, device=dev)
            best = None
            for _ in range(3):
                assert lib.walk_probe(ctypes.c_void_p(src.data_ptr()), L, ctypes.c_void_p(lst.data_ptr()),
                                      ctypes.c_void_p(cnt.data_ptr()), ctypes.c_void_p(cyc.data_ptr())) == 0
                c = int(cyc.item())
                best = c if best is None else min(best, c)
            n = int(cnt.item())
            want = host_chain(bytes(src.cpu().numpy().tobytes()))
            got = [(int(v) & 0xFFFF, (int(v) >> 16) & 0xFFFF) for v in lst[:n].cpu().numpy().astype(np.uint32)]
            ok = got == [(p, d & 0xFFFF) for p, d in want]
            rows.append({"dist": dist, "page": i, "bytes": L, "tokens": n, "cycles": best,
                         "cyc_per_token": round(best / max(n, 1), 1), "ok": ok})
            print(json.dumps(rows[-1]), flush=True)
    tot_c = sum(r["cycles"] for r in rows)
    tot_t = sum(r["tokens"] for r in rows)
    print(json.dumps({"summary": True, "cyc_per_token": round(tot_c / tot_t, 2),
                      "all_ok": all(r["ok"] for r in rows)}), flush=True)


if __name__ == "__main__":
    main()
