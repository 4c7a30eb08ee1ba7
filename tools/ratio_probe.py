"""Diagnostic: compressed bytes of the device encoders against the reference's own encoders
(oracle/_ref, the vendored LZ4 1.7.5 / zstd 1.1.2 / zlib 1.2.8 at level 1) on the parity suite's
page sets, per codec, distribution and page size.  Prints one JSON line per case; the bounds the
parity tests assert (tests/test_gpu_*.py, "ratio pins") come from these numbers.

    python tools/ratio_probe.py > gpurun_out/ratio_probe.jsonl
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402  (checker only: the reference's encoders size the pages)
from tyche_amd import _lib, codec  # noqa: E402

LZ4, ZLIB, ZSTD = 1, 2, 3
DEV = torch.device("cuda:0")
# the seeds and first-page numbers of the round-trip tests (test_gpu_lz4/zstd/zlib)
CASES = {LZ4: (48, 4242), ZSTD: (32, 777), ZLIB: (32, 31337)}
REF = {LZ4: O.ref_lz4_compress, ZSTD: O.ref_zstd_compress, ZLIB: O.ref_zlib_compress}
NAME = {LZ4: "lz4", ZSTD: "zstd", ZLIB: "zlib"}


def main():
    assert O.have_ref(), "oracle/_ref is needed (the reference's encoders)"
    # zstd: the multi-pass encoder on every batch size, as in tests/test_gpu_zstd.py (its autouse
    # fixture) and at the bench's 1M pages; below 4,096 pages the one-launch kernel would run
    _lib.set_knob("ZSTD_SPLIT_MIN", 1)
    for cid in (LZ4, ZSTD, ZLIB):
        n, seed = CASES[cid]
        for plen in (8192, 16384, 32768):
            for dist in range(6):
                pages = codec.pagegen(n, plen, seed=seed, first=plen + dist * 100, dist=dist, device=DEV)
                _, clen = codec.compress_pages(pages, compressor_id=cid)
                torch.cuda.synchronize()
                host = pages.cpu().numpy()
                gpu = int(clen.to(torch.int64).sum())
                ref = sum(len(REF[cid](host[i].tobytes())) for i in range(n))
                print(json.dumps({"codec": NAME[cid], "plen": plen, "dist": dist, "n": n, "gpu_bytes": gpu,
                                  "ref_bytes": ref, "gpu_over_ref": round(gpu / ref, 4),
                                  "ratio_gpu": round(n * plen / gpu, 4), "ratio_ref": round(n * plen / ref, 4)}),
                      flush=True)


if __name__ == "__main__":
    main()
