"""Writes the reference's 60 sample_data pages, rebuilt from tests/golden/lz4_sample.npz
(decoded by the oracle, checked by SHA-256), under the directory given (default
gpurun_out/sample_data) -- for running the reference app on the GPU box, where
/root/reference does not exist."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main(out):
    g = np.load(os.path.join(ROOT, "tests", "golden", "lz4_sample.npz"), allow_pickle=False)
    for i, name in enumerate(g["names"]):
        comp = g["comp"][g["comp_off"][i]:g["comp_off"][i] + g["comp_len"][i]]
        r, page = O.lz4_decompress(comp, int(g["size"][i]))
        assert r == g["size"][i] and hashlib.sha256(page).digest() == g["digest"][i].tobytes(), name
        path = os.path.join(out, str(name))
        os.makedirs(os.path.dirname(path), exist_ok=True)
        open(path, "wb").write(page)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "sample_data"))
