"""Diagnostic: time compress/decompress of one codec for several library builds
(ablation or tuning variants), one child process per library, no correctness
assertions (ablation builds produce wrong output by design).

    TYCHE_LIBS=a.so,b.so CODEC=zstd PLEN=32768 PAGES=131072 python tools/time_variant.py
"""
import os
import subprocess
import sys

CHILD = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
from tyche_amd import codec
ids = {"lz4": 1, "zlib": 2, "zstd": 3}
cid = ids[os.environ.get("CODEC", "lz4")]
n = int(os.environ.get("PAGES", "131072")); plen = int(os.environ.get("PLEN", "16384"))
pages = codec.pagegen(n, plen, dist=int(os.environ.get("DIST", "0")))
comp, clen = codec.compress_pages(pages, compressor_id=cid)
torch.cuda.synchronize()
mx = int(clen.max())
out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=cid, max_comp_len=mx)
torch.cuda.synchronize()
ok = bool((rv == plen).all()) and torch.equal(out, pages)
# digest of the first 4,096 compressed pages (bytes past each page's length masked): variants that
# must produce the same streams print the same digest
import hashlib
k = min(n, 4096)
mask = torch.arange(comp.shape[1], device=comp.device)[None, :] < clen[:k, None].to(torch.int64)
dig = hashlib.sha1((comp[:k] * mask).cpu().numpy().tobytes() + clen[:k].cpu().numpy().tobytes()).hexdigest()[:12]
def t(fn, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); best = min(best, e0.elapsed_time(e1))
    return best
d = t(lambda: codec.decompress_pages(comp, clen, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx))
c = t(lambda: codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen))
print(f"{os.path.basename(os.environ['TYCHE_CODEC_LIB'])}: compress {c * (1 << 20) / n:8.1f} ms/1M  "
      f"decompress {d * (1 << 20) / n:8.1f} ms/1M  ratio {n * plen / float(clen.to(torch.int64).sum()):.4f}  correct={ok}  streams {dig}")
'''


def main():
    for lib in os.environ.get("TYCHE_LIBS", "tyche_amd/libtyche_codec.so").split(","):
        env = dict(os.environ, TYCHE_CODEC_LIB=lib)
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=900)
        print(r.stdout.strip() or r.stderr.strip()[-800:], flush=True)


if __name__ == "__main__":
    main()
