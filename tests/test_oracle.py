"""The CPU oracle (oracle/lz4_oracle.c) pinned against the reference's outputs.

Fixtures in tests/golden/ were produced by oracle/gen_golden.py from the
reference's own vendored LZ4 1.7.5 (src/lz4/lz4.c) compiled here.  The KAT is
src/tests.c:342-378 (4096-byte Lorem text; LZ4 level 1 -> 2578 bytes).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import ROOT, load_golden, unpack


def test_kat_lorem_exact(oracle_mod):
    O = oracle_mod
    g = load_golden("kat_lorem.npz")
    text = g["text"].tobytes()
    assert len(text) == 4096
    comp = O.lz4_compress(text)
    assert len(comp) == 2578
    assert comp == g["lz4"].tobytes()
    rv, out = O.lz4_decompress(comp, len(text))
    assert rv == 4096 and out == text
    assert len(g["zlib"]) == 1759 and len(g["zstd"]) == 1709


def test_generated_pages_exact(oracle_mod):
    O = oracle_mod
    g = load_golden("lz4_generated.npz")
    seed = int(g["seed"])
    for i, (dist, plen, idx) in enumerate(g["meta"]):
        page = O.pagegen(1, int(plen), seed=seed, first=int(idx), dist=int(dist))[0].tobytes()
        assert hashlib.sha256(page).digest() == g["digest"][i].tobytes(), "page generator drifted"
        ref = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        assert O.lz4_compress(page) == ref, (dist, plen, idx)
        rv, out = O.lz4_decompress(ref, int(plen))
        assert rv == plen and out == page


def test_sample_pages_exact(oracle_mod):
    O = oracle_mod
    g = load_golden("lz4_sample.npz")
    for i in range(len(g["names"])):
        comp = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        rv, out = O.lz4_decompress(comp, int(g["size"][i]))
        assert rv == g["size"][i]
        assert hashlib.sha256(out).digest() == g["digest"][i].tobytes()
    for k, i in enumerate(g["raw_index"]):
        raw = unpack(g["raw"], g["raw_off"], g["raw_len"], k)
        assert O.lz4_compress(raw) == unpack(g["comp"], g["comp_off"], g["comp_len"], int(i))


def test_malformed_streams(oracle_mod):
    O = oracle_mod
    g = load_golden("lz4_malformed.npz")
    for i in range(len(g["cap"])):
        s = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        rv, out = O.lz4_decompress(s, int(g["cap"][i]))
        assert rv == g["rv"][i], (i, s[:16], g["cap"][i])
        if g["defined"][i]:
            assert hashlib.sha256(out).digest() == g["digest"][i].tobytes()


def test_compress_limited_output(oracle_mod):
    """cap < bound selects limitedOutput (lz4.c:671-675): 0 when it does not fit, else the same bytes."""
    O = oracle_mod
    page = O.pagegen(1, 16384, dist=0)[0].tobytes()
    full = O.lz4_compress(page)
    assert O.lz4_compress(page, cap=len(full)) == full
    assert O.lz4_compress(page, cap=len(full) - 1) == b""
    rnd = O.pagegen(1, 4096, dist=4)[0].tobytes()
    assert O.lz4_compress(rnd, cap=4096) == b""


@pytest.mark.parametrize("n", [0, 1, 5, 12, 13, 14, 100])
def test_tiny_inputs(oracle_mod, n):
    O = oracle_mod
    data = bytes((i * 7) & 0xFF for i in range(n))
    comp = O.lz4_compress(data)
    assert len(comp) == 1 + n if n < 13 else len(comp) > 0
    rv, out = O.lz4_decompress(comp, n)
    assert rv == n and out == data


def test_against_reference_build_random(oracle_mod):
    """Randomised cross-check with the reference build (only where oracle/_ref exists)."""
    O = oracle_mod
    if not O.have_ref():
        pytest.skip("oracle/_ref/libtyche_ref.so not built (no /root/reference here)")
    rng = np.random.default_rng(7)
    pages = O.pagegen(24, 8192, seed=99, dist=0)
    for t in range(120):
        kind = t % 4
        if kind == 0:
            data = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
        elif kind == 1:
            data = (rng.integers(0, 4, int(rng.integers(1, 5000)), dtype=np.uint8) * 17).tobytes()
        else:
            p = bytearray(pages[t % 24].tobytes()[: int(rng.integers(1, 8192))])
            for _ in range(int(rng.integers(0, 20))):
                if p:
                    p[int(rng.integers(0, len(p)))] = int(rng.integers(0, 256))
            data = bytes(p)
        ref = O.ref_lz4_compress(data)
        assert O.lz4_compress(data) == ref
        # corrupt and compare decoder verdicts
        s = bytearray(ref)
        for _ in range(int(rng.integers(0, 3))):
            if s:
                s[int(rng.integers(0, len(s)))] = int(rng.integers(0, 256))
        cap = len(data) + int(rng.integers(-3, 4))
        cap = max(cap, 0)
        r1, o1 = O.lz4_decompress(bytes(s), cap)
        r2, o2 = O.ref_lz4_decompress(bytes(s), cap)
        assert r1 == r2


# ----------------------------------------------------------------- zlib (A11)
def test_zlib_kat(oracle_mod):
    """src/tests.c:384-413: zlib level 1 of the Lorem KAT is 1759 bytes and inflates back."""
    O = oracle_mod
    g = load_golden("kat_lorem.npz")
    rv, out = O.zlib_uncompress(g["zlib"].tobytes(), 4096)
    assert rv == 4096 and out == g["text"].tobytes()
    assert O.adler32(out) == int.from_bytes(g["zlib"].tobytes()[-4:], "big")


def test_zlib_streams_exact(oracle_mod):
    """Stored (level 0), fixed and dynamic-Huffman blocks produced by the reference's compress2."""
    O = oracle_mod
    g = load_golden("zlib_streams.npz")
    for i in range(len(g["labels"])):
        s = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        n = int(g["size"][i])
        rv, out = O.zlib_uncompress(s, n)
        assert rv == n, (g["labels"][i], g["level"][i], rv)
        assert hashlib.sha256(out).digest() == g["digest"][i].tobytes()


def test_zlib_malformed(oracle_mod):
    """Reference uncompress() verdicts, exactly: success with length and bytes, and on failure the
    same code -- Z_DATA_ERROR(-3) or Z_BUF_ERROR(-5), which uncompress() picks from inflate's state
    when the output fills (uncompr.c:47-53: Z_BUF_ERROR with all input consumed becomes
    Z_DATA_ERROR).  buffer__decompress maps both to E_BUFFER_DECOMPRESSION_PROBLEM
    (src/buffer.c:257-260), but the oracle and the device decoders reproduce the split."""
    O = oracle_mod
    g = load_golden("zlib_malformed.npz")
    for i in range(len(g["cap"])):
        s = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        rv, out = O.zlib_uncompress(s, int(g["cap"][i]))
        want = int(g["rv"][i])
        assert rv == want, (i, rv, want)
        if want >= 0:
            assert hashlib.sha256(out).digest() == g["digest"][i].tobytes()


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libtyche_ref.so")),
                    reason="oracle/_ref (the reference's own zlib, built from /root/reference) not present")
def test_zlib_seeded_corruptions_vs_reference(oracle_mod):
    """1,500 seeded corruptions of reference-compressed pages (bit flips, truncations, byte stores,
    short capacities): the oracle's code and bytes equal the reference build's uncompress() on
    every one, Z_BUF_ERROR / Z_DATA_ERROR included."""
    O = oracle_mod
    rng = np.random.default_rng(5)
    pages = O.pagegen(50, 16384, seed=3)
    for i in range(50):
        base = O.ref_zlib_compress(pages[i].tobytes())
        for t in range(30):
            b = bytearray(base)
            mode, cap = t % 4, 16384
            if mode == 0:
                for _ in range(int(rng.integers(1, 4))):
                    b[int(rng.integers(len(b)))] ^= 1 << int(rng.integers(8))
            elif mode == 1:
                b = b[:int(rng.integers(1, len(b)))]
            elif mode == 2:
                b[int(rng.integers(len(b)))] = int(rng.integers(256))
            else:
                cap = int(rng.integers(1, 16384))
            r1, o1 = O.zlib_uncompress(bytes(b), cap)
            r2, o2 = O.ref_zlib_uncompress(bytes(b), cap)
            assert r1 == r2, (i, t, r1, r2)
            if r1 >= 0:
                assert o1 == o2, (i, t)


# ----------------------------------------------------------------- zstd (A9)
def test_zstd_kat(oracle_mod):
    """src/tests.c:415-436: zstd level 1 of the Lorem KAT is 1709 bytes and decodes back."""
    O = oracle_mod
    g = load_golden("kat_lorem.npz")
    rv, out = O.zstd_decompress(g["zstd"].tobytes(), 4096)
    assert rv == 4096 and out == g["text"].tobytes()


def test_zstd_streams_exact(oracle_mod):
    """Reference ZSTD_compress frames at levels 1/3/9/19, multi-block ZSTD_compressContinue
    frames and XXH64-checksummed frames decode to the original bytes."""
    O = oracle_mod
    g = load_golden("zstd_streams.npz")
    kinds = set()
    for i in range(len(g["labels"])):
        s = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        n = int(g["size"][i])
        rv, out = O.zstd_decompress(s, n)
        assert rv == n, (g["labels"][i], g["level"][i], rv)
        assert hashlib.sha256(out).digest() == g["digest"][i].tobytes()
        kinds.add(s[4])   # frame header descriptors seen
    assert len(kinds) >= 3


def test_zstd_malformed(oracle_mod):
    """Reference ZSTD_decompress verdicts on corrupted / truncated / short-capacity frames:
    error where the reference errs (buffer.c:264-266 only tests ZSTD_isError), otherwise the
    same size and bytes -- including frames whose corruption the reference does not detect."""
    O = oracle_mod
    g = load_golden("zstd_malformed.npz")
    for i in range(len(g["cap"])):
        s = unpack(g["comp"], g["comp_off"], g["comp_len"], i)
        rv, out = O.zstd_decompress(s, int(g["cap"][i]))
        want = int(g["rv"][i])
        if want >= 0:
            assert rv == want, (i, rv, want)
            assert hashlib.sha256(out).digest() == g["digest"][i].tobytes()
        else:
            assert rv < 0, (i, rv, want)


def test_zstd_xxh64_known_answer(oracle_mod):
    """XXH64 of the empty input with seed 0 (published xxHash test vector)."""
    assert oracle_mod.xxh64(b"") == 0xEF46DB3751D8E999
