"""Diagnostic: knob A/B of one codec's device compress -- time and ratio per setting, one child process each.

    CODEC=lz4 PLEN=16384 PAGES=262144 python tools/knob_ab.py base LZ4_ENC_WAVES=3,LZ4_ENC_SEED=8192

Each argument is a comma-separated list of NAME=VALUE engine knobs (TYCHE_NAME in the child's environment;
"base" sets none).  The round trip through the device decoder is checked once per setting.
"""
import os, subprocess, sys
CHILD = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
from tyche_amd import codec
n = int(os.environ.get("PAGES", "262144")); plen = int(os.environ.get("PLEN", "16384"))
cid = {"lz4": 1, "zlib": 2, "zstd": 3}[os.environ.get("CODEC", "lz4")]
pages = codec.pagegen(n, plen)
comp, clen = codec.compress_pages(pages, compressor_id=cid)
torch.cuda.synchronize()
mx = int(clen.max())
out, rv = codec.decompress_pages(comp, clen, plen, compressor_id=cid, max_comp_len=mx)
torch.cuda.synchronize()
ok = bool((rv == plen).all()) and torch.equal(out, pages)
def t(fn, reps=4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); best = min(best, e0.elapsed_time(e1))
    return best
c = t(lambda: codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen))
print(f"{os.environ.get('TAG','')}: compress {c * (1 << 20) / n:7.2f} ms/1M ratio {n * plen / float(clen.to(torch.int64).sum()):.4f} correct={ok}")
'''
for spec in sys.argv[1:]:
    env = dict(os.environ, TAG=spec)
    for kv in spec.split(","):
        if "=" in kv:
            k, v = kv.split("="); env["TYCHE_" + k] = v
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
    print(r.stdout.strip() or r.stderr.strip()[-800:], flush=True)
