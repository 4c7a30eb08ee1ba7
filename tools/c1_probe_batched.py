"""Diagnostic: one run of integration/_app/tyche_batched on 256 synthetic pages, full output kept.

    python tools/c1_probe_batched.py [workers] [mem] [codec]   ->  gpurun_out/c1_probe_batched.{out,err}
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

workers = sys.argv[1] if len(sys.argv) > 1 else "16"
mem = sys.argv[2] if len(sys.argv) > 2 else "1000000"
codec = sys.argv[3] if len(sys.argv) > 3 else "lz4"
d = tempfile.mkdtemp()
os.makedirs(os.path.join(d, "16k"))
pages = O.pagegen(256, 16384)
for i in range(256):
    with open(os.path.join(d, "16k", f"page{i:04d}"), "wb") as f:
        f.write(pages[i].tobytes())
env = dict(os.environ, TYCHE_APP_WATCHDOG="15", TYCHE_LOG_ERRORS="1")
app = os.path.join(ROOT, "integration", "_app", "tyche_batched")
p = subprocess.run([app, "-c", codec, "-p", os.path.join(d, "16k"), "-w", workers, "-d", "3", "-m", mem, "-f", "20"],
                   stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=90, env=env)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
open(os.path.join(ROOT, "gpurun_out", "c1_probe_batched.out"), "wb").write(p.stdout)
open(os.path.join(ROOT, "gpurun_out", "c1_probe_batched.err"), "wb").write(p.stderr)
print("rc", p.returncode)
