"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY.

Generates the committed parity fixtures in tests/golden/ from the REFERENCE's
own vendored codecs (LZ4 1.7.5 / zlib 1.2.8 / zstd 1.1.2 compiled from
/root/reference/src by oracle/Makefile into oracle/_ref/libtyche_ref.so).
Run here, where /root/reference exists:

    make -C oracle ref && python oracle/gen_golden.py

Fixtures (all data, no reference source):
  kat_lorem.npz       the 4096-byte KAT input of src/tests.c:342-378 and its
                      LZ4 / zlib-1 / zstd-1 encodings (2578 / 1759 / 1709 B)
  lz4_generated.npz   reference LZ4 encodings of repo-generated pages
                      (pagegen.h, every distribution, 8/16/32 KiB) + input digests
  lz4_sample.npz      reference LZ4 encodings of the 60 sample_data pages, the
                      SHA-256 of each original, and 6 originals in full
  lz4_malformed.npz   corrupted / truncated / random streams with the reference
                      LZ4_decompress_safe return value (and output digest when
                      the output is defined)
  zlib_streams.npz    reference compress2 encodings (levels 0/1/6/9: stored,
                      fixed and dynamic blocks) of generated pages, sample pages
                      and short inputs, with the input digests
  zlib_malformed.npz  corrupted / truncated / short-capacity zlib streams with the
                      reference uncompress() result (Z_OK length or error code)
  zstd_streams.npz    reference ZSTD_compress frames (levels 1/3/9/19: raw, RLE and
                      Huffman 1X/4X literals, predefined / RLE / FSE-compressed
                      sequence tables), multi-block frames from ZSTD_compressContinue
                      (no content size, set_repeat tables, carried repeat offsets)
                      and frames with an XXH64 content checksum, with input digests
  zstd_malformed.npz  corrupted / truncated / short-capacity frames with the
                      reference ZSTD_decompress result (size, or -1 for ZSTD_isError)
                      and the output digest when it succeeds
"""
from __future__ import annotations

import glob
import hashlib
import os
import re
import sys

import numpy as np

sys.path[0] = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
REF = "/root/reference"
SEED = 20170303


def sha(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def pack(blobs: list[bytes]):
    lens = np.array([len(b) for b in blobs], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    data = np.frombuffer(b"".join(blobs), dtype=np.uint8) if blobs else np.zeros(0, np.uint8)
    return data, offs, lens


def kat_text() -> bytes:
    s = open(os.path.join(REF, "src", "tests.c")).read()
    i = s.index("void tests__compression")
    j = s.index("int src_size", i)
    return "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', s[i:j])).encode()


def gen_kat():
    t = kat_text()
    assert len(t) == 4096
    lz4 = O.ref_lz4_compress(t)
    zl = O.ref_zlib_compress(t, 1)
    zs = O.ref_zstd_compress(t, 1)
    print("KAT", len(lz4), len(zl), len(zs))
    np.savez_compressed(os.path.join(OUT, "kat_lorem.npz"), text=np.frombuffer(t, np.uint8),
                        lz4=np.frombuffer(lz4, np.uint8), zlib=np.frombuffer(zl, np.uint8),
                        zstd=np.frombuffer(zs, np.uint8))


def gen_generated():
    rows = []   # (dist, page_len, index)
    comps, digests = [], []
    for dist in range(6):
        for plen in (8192, 16384, 32768):
            n = 1 if dist == 4 else 3
            first = 1000 * dist + plen // 1024
            pages = O.pagegen(n, plen, seed=SEED, first=first, dist=dist)
            for k in range(n):
                p = pages[k].tobytes()
                c = O.ref_lz4_compress(p)
                r, out = O.ref_lz4_decompress(c, plen)
                assert r == plen and out == p
                rows.append((dist, plen, first + k))
                comps.append(c)
                digests.append(sha(p))
    data, offs, lens = pack(comps)
    np.savez_compressed(os.path.join(OUT, "lz4_generated.npz"), seed=np.int64(SEED),
                        meta=np.array(rows, dtype=np.int64), comp=data, comp_off=offs, comp_len=lens,
                        digest=np.frombuffer(b"".join(digests), np.uint8).reshape(-1, 32))
    print("generated", len(rows), data.size)


def gen_sample():
    files = sorted(glob.glob(os.path.join(REF, "sample_data", "*", "*", "*", "*")))
    names, comps, digests, sizes = [], [], [], []
    raw_keep = []
    for f in files:
        p = open(f, "rb").read()
        c = O.ref_lz4_compress(p)
        rel = os.path.relpath(f, os.path.join(REF, "sample_data"))
        names.append(rel)
        comps.append(c)
        digests.append(sha(p))
        sizes.append(len(p))
    # keep a table page and an index page of each size in full (compress parity inputs)
    keep = []
    for sz in ("8k", "16k", "32k"):
        for kind in ("tables", "indexes"):
            idx = [i for i, n in enumerate(names) if n.startswith(sz + "/") and f"/{kind}/" in n][0]
            keep.append(idx)
            raw_keep.append(open(os.path.join(REF, "sample_data", names[idx]), "rb").read())
    data, offs, lens = pack(comps)
    rdata, roffs, rlens = pack(raw_keep)
    np.savez_compressed(os.path.join(OUT, "lz4_sample.npz"), names=np.array(names), comp=data, comp_off=offs,
                        comp_len=lens, digest=np.frombuffer(b"".join(digests), np.uint8).reshape(-1, 32),
                        size=np.array(sizes, np.int64), raw_index=np.array(keep, np.int64), raw=rdata,
                        raw_off=roffs, raw_len=rlens)
    print("sample", len(names), data.size, rdata.size)


def reads_unwritten(s: bytes, cap: int) -> bool:
    """True if the stream has a match with offset 0 before it ends or fails.

    Such a match copies bytes the reference never wrote (whatever its 8-byte
    wild copies left in the output buffer, lz4.c:1158, 1209-1236), so the
    decoded bytes are an artefact of the implementation; only the return value
    is a parity target for these streams."""
    ip, op, L = 0, 0, len(s)
    while ip < L:
        t = s[ip]
        ip += 1
        lit = t >> 4
        if lit == 15:
            while True:
                x = s[ip] if ip < L else 0
                ip += 1
                lit += x
                if not (ip < L - 15 and x == 255):
                    break
        if op + lit > cap - 12 or ip + lit > L - 8:
            return False
        ip += lit
        op += lit
        off = s[ip] | (s[ip + 1] << 8)
        ip += 2
        if off > op:
            return False
        if off == 0:
            return True
        ml = t & 15
        if ml == 15:
            while True:
                x = s[ip]
                ip += 1
                if ip > L - 5:
                    return False
                ml += x
                if x != 255:
                    break
        ml += 4
        if op + ml > cap - 5:
            return False
        op += ml
    return False


def gen_malformed():
    rng = np.random.default_rng(SEED)
    cases = []   # (stream, out_cap)
    base_pages = O.pagegen(4, 16384, seed=SEED, first=777, dist=0)
    streams = [O.ref_lz4_compress(p.tobytes()) for p in base_pages]
    small = O.ref_lz4_compress(kat_text())
    streams.append(small)
    for s in streams:
        n = len(s)
        for cut in sorted(set([1, 2, 3, 5, 8, 13, n // 3, n // 2, n - 9, n - 6, n - 5, n - 1])):
            if 0 < cut < n:
                cases.append((s[:cut], 16384))
        for _ in range(12):
            b = bytearray(s)
            for _ in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, n))] = int(rng.integers(0, 256))
            cases.append((bytes(b), 16384 if len(s) > 3000 else 4096))
        cases.append((s, 16383))         # output one byte short
        cases.append((s, 16384 + 100))   # larger capacity: decode stops at the stream end
        cases.append((s + b"\x00", 16384))   # trailing garbage
    for _ in range(40):
        ln = int(rng.integers(1, 300))
        cases.append((rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), int(rng.choice([64, 1024, 16384]))))
    # hand-made edge cases
    cases += [
        (b"\x00", 0), (b"\x00", 1), (b"\x10A", 0), (b"\x10A", 1), (b"\xf0", 64), (b"\xf0\xff", 64),
        (b"\x50hello", 5), (b"\x50hello", 4), (b"\x50hello", 64),
        (b"\x1fa\x01\x00\xff\xff\x00" + b"\x50abcde", 600),      # long RLE match then literals
        (b"\x1fa\x00\x00\x05" + b"\x50abcde", 64),                 # offset 0
        (b"\x14a\x02\x00" + b"\x50abcde", 64),                     # offset beyond output
        (b"\x4fabcd\x04\x00\x10" + b"\x50abcde", 64),              # overlap offset 4
        (b"\x80abcdefgh" + b"\x00", 8),
    ]
    streams_out, caps, rvs, digs, defined = [], [], [], [], []
    for s, cap in cases:
        r0, o0 = O.ref_lz4_decompress(s, cap, fill=0)
        r1, o1 = O.ref_lz4_decompress(s, cap, fill=0xFF)
        assert r0 == r1
        streams_out.append(s)
        caps.append(cap)
        rvs.append(r0)
        ok = r0 >= 0 and o0 == o1 and not reads_unwritten(s, cap)
        defined.append(ok)
        digs.append(sha(o0) if ok else b"\0" * 32)
    data, offs, lens = pack(streams_out)
    np.savez_compressed(os.path.join(OUT, "lz4_malformed.npz"), comp=data, comp_off=offs, comp_len=lens,
                        cap=np.array(caps, np.int64), rv=np.array(rvs, np.int64),
                        defined=np.array(defined, bool),
                        digest=np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 32))
    print("malformed", len(cases), "errors", sum(r < 0 for r in rvs), "undefined", sum(not d for d in defined))


def zlib_inputs():
    """(label, bytes) inputs for the zlib fixtures."""
    out = []
    for dist in range(6):
        for plen in (8192, 16384, 32768):
            first = 5000 + 1000 * dist + plen // 1024
            out.append((f"gen/{dist}/{plen}/{first}", O.pagegen(1, plen, seed=SEED, first=first, dist=dist)[0].tobytes()))
    files = sorted(glob.glob(os.path.join(REF, "sample_data", "*", "*", "*", "*")))
    for f in files[::3]:
        out.append(("sample/" + os.path.relpath(f, os.path.join(REF, "sample_data")), open(f, "rb").read()))
    out.append(("kat", kat_text()))
    for n in (0, 1, 2, 3, 7, 64, 300):
        out.append((f"short/{n}", bytes((i * 37 + 11) & 0xFF for i in range(n))))
    out.append(("short/hello", b"hello hello hello hello"))
    return out


def gen_zlib_streams():
    labels, levels, comps, digests, sizes = [], [], [], [], []
    for label, data in zlib_inputs():
        for level in (0, 1, 6, 9):
            if level != 1 and not (label.startswith("gen/0/16384") or label.startswith("short") or label == "kat"):
                continue
            c = O.ref_zlib_compress(data, level)
            r, out = O.ref_zlib_uncompress(c, len(data))
            assert r == len(data) and out == data
            labels.append(label)
            levels.append(level)
            comps.append(c)
            digests.append(sha(data))
            sizes.append(len(data))
    data, offs, lens = pack(comps)
    np.savez_compressed(os.path.join(OUT, "zlib_streams.npz"), seed=np.int64(SEED), labels=np.array(labels),
                        level=np.array(levels, np.int64), comp=data, comp_off=offs, comp_len=lens,
                        size=np.array(sizes, np.int64),
                        digest=np.frombuffer(b"".join(digests), np.uint8).reshape(-1, 32))
    print("zlib streams", len(labels), data.size)


def gen_zlib_malformed():
    rng = np.random.default_rng(SEED + 2)
    cases = []   # (stream, out_cap)
    srcs = [O.pagegen(1, 16384, seed=SEED, first=9000 + k, dist=k % 4)[0].tobytes() for k in range(3)]
    srcs.append(kat_text())
    srcs.append(b"hello hello hello hello")
    streams = [O.ref_zlib_compress(d, 1) for d in srcs] + [O.ref_zlib_compress(srcs[0][:3000], 0)]
    sizes = [len(d) for d in srcs] + [3000]
    for s, n_out in zip(streams, sizes):
        n = len(s)
        for cut in sorted(set([1, 2, 3, 5, 9, n // 3, n // 2, n - 5, n - 4, n - 1])):
            if 0 < cut < n:
                cases.append((s[:cut], n_out))
        for _ in range(14):
            b = bytearray(s)
            for _ in range(int(rng.integers(1, 3))):
                b[int(rng.integers(0, n))] ^= 1 << int(rng.integers(0, 8))
            cases.append((bytes(b), n_out))
        cases.append((s, n_out - 1))           # output one byte short
        cases.append((s, n_out + 100))         # larger capacity (Z_OK with the true length)
        cases.append((s + b"\x00\x00", n_out))   # trailing bytes after the adler32
    for _ in range(30):
        ln = int(rng.integers(1, 200))
        cases.append((rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), 4096))
    for _ in range(10):   # valid header, random body
        ln = int(rng.integers(1, 200))
        cases.append((b"\x78\x01" + rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), 4096))
    cases += [
        (b"", 16), (b"\x78", 16), (b"\x78\x01", 16), (b"\x78\x02", 16), (b"\x79\x01", 16),
        (b"\x78\xbb\x00\x00\x00\x00", 16),                      # FDICT
        (b"\x78\x01\x01\x00\x00\xff\xff\x00\x00\x00\x01", 16),  # empty stored block, adler 1
        (b"\x78\x01\x01\x01\x00\xfe\xff\x41\x00\x42\x00\x42", 16),  # stored 'A'
        (b"\x78\x01\x01\x01\x00\xfe\xfe\x41\x00\x42\x00\x42", 16),  # bad NLEN
        (b"\x78\x01\x07", 16),                                  # reserved block type
    ]
    streams_out, caps, rvs, digs = [], [], [], []
    for s, cap in cases:
        r, out = O.ref_zlib_uncompress(s, cap)
        streams_out.append(s)
        caps.append(cap)
        rvs.append(r)
        digs.append(sha(out) if r >= 0 else b"\0" * 32)
    data, offs, lens = pack(streams_out)
    np.savez_compressed(os.path.join(OUT, "zlib_malformed.npz"), comp=data, comp_off=offs, comp_len=lens,
                        cap=np.array(caps, np.int64), rv=np.array(rvs, np.int64),
                        digest=np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 32))
    print("zlib malformed", len(cases), "errors", sum(r < 0 for r in rvs))


def with_checksum(frame: bytes, content: bytes) -> bytes:
    """Sets the Content_Checksum_flag of a frame and appends XXH64(content) low 32 bits
    (the layout ZSTD_compressEnd writes, zstd_compress.c:2638-2674); the hash comes
    from the reference build's ZSTD_XXH64."""
    b = bytearray(frame)
    b[4] |= 0x04
    return bytes(b) + (O.ref_xxh64(content) & 0xFFFFFFFF).to_bytes(4, "little")


def zstd_cases():
    """(label, level, frame, content) for zstd_streams.npz."""
    out = []
    for label, data in zlib_inputs():
        levels = (1,) if not (label.startswith("gen/") or label == "kat" or label.startswith("short")) else (1, 3, 9, 19)
        for level in levels:
            out.append((label, level, O.ref_zstd_compress(data, level), data))
        if label.startswith("gen/0/") or label.startswith("gen/3/") or label == "kat":
            for chunk in (4096, 1500):
                if len(data) > chunk:
                    out.append((label + f"/blocks{chunk}", 1, O.ref_zstd_compress_blocks(data, chunk, 1), data))
        if label.startswith("gen/1/") or label == "kat":
            out.append((label + "/xxh64", 1, with_checksum(O.ref_zstd_compress(data, 1), data), data))
    return out


def gen_zstd_streams():
    labels, levels, comps, digests, sizes = [], [], [], [], []
    for label, level, c, data in zstd_cases():
        r, out = O.ref_zstd_decompress(c, len(data))
        assert r == len(data) and out == data, label
        labels.append(label)
        levels.append(level)
        comps.append(c)
        digests.append(sha(data))
        sizes.append(len(data))
    data, offs, lens = pack(comps)
    np.savez_compressed(os.path.join(OUT, "zstd_streams.npz"), seed=np.int64(SEED), labels=np.array(labels),
                        level=np.array(levels, np.int64), comp=data, comp_off=offs, comp_len=lens,
                        size=np.array(sizes, np.int64),
                        digest=np.frombuffer(b"".join(digests), np.uint8).reshape(-1, 32))
    print("zstd streams", len(labels), data.size)


def gen_zstd_malformed():
    rng = np.random.default_rng(SEED + 3)
    cases = []   # (frame, out_cap)
    srcs = [O.pagegen(1, 16384, seed=SEED, first=9100 + k, dist=k % 4)[0].tobytes() for k in range(3)]
    srcs.append(kat_text())
    frames = [O.ref_zstd_compress(d, 1) for d in srcs] + [O.ref_zstd_compress(srcs[0], 19),
                                                          O.ref_zstd_compress_blocks(srcs[1], 1500, 1),
                                                          with_checksum(O.ref_zstd_compress(srcs[3], 1), srcs[3])]
    sizes = [len(d) for d in srcs] + [len(srcs[0]), len(srcs[1]), len(srcs[3])]
    for s, n_out in zip(frames, sizes):
        n = len(s)
        for cut in sorted(set([1, 4, 5, 8, 9, 12, n // 3, n // 2, n - 5, n - 4, n - 1])):
            if 0 < cut < n:
                cases.append((s[:cut], n_out))
        for _ in range(24):
            b = bytearray(s)
            for _ in range(int(rng.integers(1, 3))):
                b[int(rng.integers(0, n))] ^= 1 << int(rng.integers(0, 8))
            cases.append((bytes(b), n_out))
        for _ in range(8):
            b = bytearray(s)
            i = int(rng.integers(0, n))
            b[i:i + 4] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
            cases.append((bytes(b[:n]), n_out))
        cases.append((s, n_out - 1))            # output one byte short
        cases.append((s, n_out + 100))          # larger capacity
        cases.append((s + b"\x00", n_out))       # trailing byte
    for _ in range(20):
        ln = int(rng.integers(1, 200))
        cases.append((rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), 4096))
    for _ in range(20):   # valid magic + single-segment header, random body
        ln = int(rng.integers(1, 200))
        cases.append((b"\x28\xb5\x2f\xfd\x20\x40" + rng.integers(0, 256, ln, dtype=np.uint8).tobytes(), 4096))
    cases += [
        (b"", 16), (b"\x28\xb5\x2f\xfd", 16), (b"\x28\xb5\x2f\xfd\x20\x00\x01\x00\x00", 16),  # empty raw block
        (b"\x28\xb5\x2f\xfd\x20\x05\x29\x00\x00hello", 16),     # raw block "hello"
        (b"\x28\xb5\x2f\xfd\x20\x07\x3b\x00\x00x", 16),         # RLE block of 7 'x'
        (b"\x28\xb5\x2f\xfd\x20\x07\x3b\x00\x00x", 6),          # RLE block too long for capacity
        (b"\x28\xb5\x2f\xfd\x28\x05\x29\x00\x00hello", 16),     # reserved FHD bit
        (b"\x28\xb5\x2f\xfd\x20\x05\x2f\x00\x00hello", 16),     # reserved block type
        (b"\x50\x2a\x4d\x18\x00\x00\x00\x00\x01\x00\x00", 16),  # skippable magic
        (b"\x28\xb5\x2f\xfd\x21\x05\x01\x29\x00\x00hello", 16),  # dictionary id
    ]
    streams_out, caps, rvs, digs = [], [], [], []
    for s, cap in cases:
        r, out = O.ref_zstd_decompress(s, cap)
        streams_out.append(s)
        caps.append(cap)
        rvs.append(r)
        digs.append(sha(out) if r >= 0 else b"\0" * 32)
    data, offs, lens = pack(streams_out)
    np.savez_compressed(os.path.join(OUT, "zstd_malformed.npz"), comp=data, comp_off=offs, comp_len=lens,
                        cap=np.array(caps, np.int64), rv=np.array(rvs, np.int64),
                        digest=np.frombuffer(b"".join(digs), np.uint8).reshape(-1, 32))
    print("zstd malformed", len(cases), "errors", sum(r < 0 for r in rvs))


if __name__ == "__main__":
    if not O.have_ref():
        sys.exit("oracle/_ref/libtyche_ref.so missing: run `make -C oracle ref` where /root/reference exists")
    os.makedirs(OUT, exist_ok=True)
    gen_kat()
    gen_generated()
    gen_sample()
    gen_malformed()
    gen_zlib_streams()
    gen_zlib_malformed()
    gen_zstd_streams()
    gen_zstd_malformed()
