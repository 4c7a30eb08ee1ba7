"""Diagnostic: time the LZ4 decode kernel of one or more library builds on the same pages.

    TYCHE_LIBS=tyche_amd/libtyche_codec.so,tyche_amd/libtyche_codec_abl1.so python tools/time_decode.py
Each library is loaded in a child process (ctypes cannot unload); prints ms per 1M pages.
"""
import os
import subprocess
import sys

CHILD = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
from tyche_amd import codec
n = int(os.environ.get("PAGES", "262144")); plen = int(os.environ.get("PLEN", "16384"))
pages = codec.pagegen(n, plen, dist=int(os.environ.get("DIST", "0")))
comp, clen = codec.compress_pages(pages)
torch.cuda.synchronize()
mx = int(clen.max())
out, rv = codec.decompress_pages(comp, clen, plen, max_comp_len=mx)
torch.cuda.synchronize()
ok = bool((rv == plen).all()) and torch.equal(out, pages)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(5):
    e0.record(); codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=mx); e1.record()
    torch.cuda.synchronize(); best = min(best, e0.elapsed_time(e1))
c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
bc = 1e9
for _ in range(3):
    c0.record(); codec.compress_pages(pages, out=comp, out_len=clen); c1.record()
    torch.cuda.synchronize(); bc = min(bc, c0.elapsed_time(c1))
ratio = n * plen / float(clen.to(torch.int64).sum())
import hashlib
ch, lh = comp[:2048].cpu().numpy(), clen[:2048].cpu().numpy()
dig = hashlib.sha1(b"".join(ch[i, :lh[i]].tobytes() for i in range(len(lh)))).hexdigest()[:12]
print(f"{os.environ['TYCHE_CODEC_LIB']}: max_comp {mx} ratio {ratio:.4f} decode {best * (1 << 20) / n:8.2f} ms/1M pages  "
      f"({n * plen / best / 1e6 / 1.073741824:7.1f} GiB/s)  encode {bc * (1 << 20) / n:8.2f} ms/1M  correct={ok}  streams {dig}")
'''


def main():
    libs = os.environ.get("TYCHE_LIBS", "tyche_amd/libtyche_codec.so").split(",")
    for lib in libs:
        env = dict(os.environ, TYCHE_CODEC_LIB=lib)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
        print(r.stdout.strip() or r.stderr.strip()[-800:], flush=True)


if __name__ == "__main__":
    main()
