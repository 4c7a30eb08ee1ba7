"""Per-section byte accounting of zstd frames (single-segment frames, RFC 8878 3.1.1).

    python tools/zstd_frame_stats.py frames.npz      # npz with 'comp' (n x slot u8) and 'clen'
    python tools/zstd_frame_stats.py --ref PAGES     # the reference's level-1 frames of bench pages

Prints, per page on average: frame bytes, literal bytes (regenerated), literal
section bytes, sequences, sequence section bytes, and the literal block types.
"""
import argparse
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def frame_stats(f):
    fhd = f[4]
    single, did, fcs_id = (fhd >> 5) & 1, fhd & 3, fhd >> 6
    pos = 5 + (0 if single else 1) + (0, 1, 2, 4)[did] + ((1 if single else 0), 2, 4, 8)[fcs_id]
    st = collections.Counter()
    while True:
        bh = f[pos] | f[pos + 1] << 8 | f[pos + 2] << 16
        last, btype, bsize = bh & 1, (bh >> 1) & 3, bh >> 3
        pos += 3
        st["blocks"] += 1
        if btype == 2:
            b = f[pos:pos + bsize]
            lt, sf = b[0] & 3, (b[0] >> 2) & 3
            if lt in (0, 1):
                hl = 1 if sf in (0, 2) else (2 if sf == 1 else 3)
                v = int.from_bytes(bytes(b[:hl]), "little")
                rs = v >> 3 if hl == 1 else v >> 4
                lsec = hl + (rs if lt == 0 else 1)
            else:
                hl = 3 if sf in (0, 1) else (4 if sf == 2 else 5)
                v = int.from_bytes(bytes(b[:hl]), "little")
                bits = (10, 10, 14, 18)[sf]
                rs = (v >> 4) & ((1 << bits) - 1)
                cs = (v >> (4 + bits)) & ((1 << bits) - 1)
                lsec = hl + cs
            st["lit_type_%d" % lt] += 1
            st["lit_bytes"] += rs
            st["lit_section"] += lsec
            s = b[lsec:]
            n = s[0]
            if n >= 255:
                n = int(s[1]) + (int(s[2]) << 8) + 0x7F00
            elif n >= 128:
                n = ((n - 128) << 8) + int(s[1])
            st["sequences"] += n
            st["seq_section"] += bsize - lsec
        else:
            st["raw_rle_block_bytes"] += bsize if btype == 0 else 1
        pos += bsize if btype != 1 else 1
        if last:
            break
    st["frame"] = len(f)
    return st


def summarize(frames, label):
    tot = collections.Counter()
    for f in frames:
        tot.update(frame_stats(bytes(f)))
    n = len(frames)
    keys = ["frame", "lit_bytes", "lit_section", "sequences", "seq_section", "blocks", "raw_rle_block_bytes"]
    print(label, " ".join(f"{k}={tot[k] / n:.1f}" for k in keys),
          " ".join(f"{k}={tot[k]}" for k in sorted(tot) if k.startswith("lit_type")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz", nargs="?")
    ap.add_argument("--ref", type=int, default=0)
    ap.add_argument("--plen", type=int, default=16384)
    a = ap.parse_args()
    if a.npz:
        z = np.load(a.npz)
        frames = [z["comp"][i, :z["clen"][i]].tobytes() for i in range(len(z["clen"]))]
        summarize(frames, "device")
    if a.ref:
        from oracle import oracle as O
        pages = O.pagegen(a.ref, a.plen, seed=11, dist=0)
        frames = [O.ref_zstd_compress_blocks(pages[i].tobytes(), a.plen, 1) for i in range(a.ref)]
        summarize(frames, "reference")


if __name__ == "__main__":
    main()
