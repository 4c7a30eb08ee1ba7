"""Diagnostic: the unchanged reference caller under TYCHE_FAIL_COMPRESS_EVERY=1 (tests/test_c1_app.py's
device-failure case), N runs, each run's exit code, wall time and stderr saved for reading.

    python tools/c1_fail_probe.py OUT_DIR [runs=4] [extra app args ...]
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402  (test infrastructure: rebuilds the sample pages)


def sample_dir():
    g = np.load(os.path.join(ROOT, "tests", "golden", "lz4_sample.npz"), allow_pickle=False)
    root = tempfile.mkdtemp(prefix="sample_data")
    for i, name in enumerate(g["names"]):
        comp = g["comp"][g["comp_off"][i]:g["comp_off"][i] + g["comp_len"][i]]
        r, page = O.lz4_decompress(comp, int(g["size"][i]))
        assert r == g["size"][i] and hashlib.sha256(page).digest() == g["digest"][i].tobytes(), name
        p = os.path.join(root, str(name))
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(page)
    return root


def main():
    out = sys.argv[1]
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    extra = sys.argv[3:]
    os.makedirs(out, exist_ok=True)
    root = sample_dir()
    app = os.path.join(ROOT, "integration", "_app", "tyche_q")
    args = ["-c", "lz4", "-p", os.path.join(root, "16k"), "-w", "1", "-d", "3", "-m", "512000", "-f", "20",
            "-U", "50"] + extra
    env = dict(os.environ, TYCHE_APP_WATCHDOG=os.environ.get("WD", "15"), TYCHE_LOG_ERRORS="1", TYCHE_FAIL_COMPRESS_EVERY="1")
    for i in range(runs):
        t0 = time.time()
        p = subprocess.run([app] + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=90, env=env)
        dt = time.time() - t0
        with open(os.path.join(out, f"run{i}.err"), "wb") as f:
            f.write(p.stderr)
        with open(os.path.join(out, f"run{i}.out"), "wb") as f:
            f.write(p.stdout)
        err = p.stderr.decode(errors="replace")
        print(json.dumps({"args": extra, "run": i, "rc": p.returncode, "s": round(dt, 1),
                          "engine_errors": err.count("tyche-engine:")}), flush=True)
        if p.returncode == -11 and os.environ.get("ALL") != "1":
            break


if __name__ == "__main__":
    main()
