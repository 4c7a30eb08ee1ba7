"""GPU parity for the gfx950 zlib inflate kernel, called through
the C ABI, against the reference's outputs and the restatement oracle.

* streams made by the reference's own compress2 (tests/golden/zlib_streams.npz:
  stored, fixed and dynamic-Huffman blocks, levels 0/1/6/9) decode bit-exactly;
* every malformed / truncated / short-capacity stream of
  tests/golden/zlib_malformed.npz gets the oracle's result exactly and the
  reference's verdict (success and length exactly; failure code up to the
  Z_BUF_ERROR / Z_DATA_ERROR split the oracle tests explain);
* streams from the host zlib (Python's zlib module: a different deflate
  implementation, all strategies) decode exactly -- they exercise long (> 10
  bit) codes, fixed blocks, RLE-only and Huffman-only parses;
* streams at every byte alignment, the Buffer API with its exact-length rule
  (src/buffer.c:257-260), and a 16K-page batch.
"""
import ctypes
import hashlib
import zlib

import numpy as np
import pytest
import torch

from conftest import load_golden, unpack

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
ZLIB = 2


@pytest.fixture(scope="module")
def tc():
    from tyche_amd import _lib, codec
    lib = _lib.load()
    assert lib.tyche_device_ready() == 1, _lib.last_error()
    return codec


def ragged_inflate(tc, streams, caps, shift=0):
    """Inflate byte strings (each placed at a 16-byte boundary + shift) into per-page capacities."""
    n = len(streams)
    lens = [len(s) for s in streams]
    offs = np.zeros(n, np.int64)
    pos = 0
    for i, s in enumerate(streams):
        offs[i] = pos + shift
        pos += (len(s) + shift + 15) // 16 * 16 + 16
    buf = np.zeros(pos + 64, np.uint8)
    for i, s in enumerate(streams):
        buf[offs[i]:offs[i] + len(s)] = np.frombuffer(s, np.uint8)
    ooffs = np.zeros(n, np.int64)
    opos = 0
    for i, c in enumerate(caps):
        ooffs[i] = opos
        opos += (c + 15) // 16 * 16 + 16
    d_stream = torch.from_numpy(buf).to(DEV)
    d_out = torch.full((opos + 64,), 0xAB, dtype=torch.uint8, device=DEV)
    d_offs = torch.from_numpy(offs).to(DEV)
    d_lens = torch.tensor(lens, dtype=torch.int32, device=DEV)
    d_caps = torch.tensor(caps, dtype=torch.int32, device=DEV)
    d_ooffs = torch.from_numpy(ooffs).to(DEV)
    d_rv = torch.empty(n, dtype=torch.int32, device=DEV)
    tc.decompress_ragged(d_stream, d_offs, d_lens, d_caps, d_out, d_ooffs, d_rv,
                         max_src_length=max(lens + [1]), max_capacity=max(caps + [0]), compressor_id=ZLIB)
    torch.cuda.synchronize()
    rv = d_rv.cpu().numpy()
    out = d_out.cpu().numpy()
    return rv, [out[ooffs[i]:ooffs[i] + max(int(rv[i]), 0)].tobytes() for i in range(n)]


def test_inflate_kat(tc):
    g = load_golden("kat_lorem.npz")
    rv, outs = ragged_inflate(tc, [g["zlib"].tobytes()], [4096])
    assert rv[0] == 4096 and outs[0] == g["text"].tobytes()


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 5])
def test_inflate_reference_streams(tc, shift):
    g = load_golden("zlib_streams.npz")
    streams = [unpack(g["comp"], g["comp_off"], g["comp_len"], i) for i in range(len(g["labels"]))]
    caps = [int(x) for x in g["size"]]
    rv, outs = ragged_inflate(tc, streams, caps, shift)
    for i in range(len(streams)):
        assert rv[i] == caps[i], (g["labels"][i], int(g["level"][i]), rv[i])
        assert hashlib.sha256(outs[i]).digest() == g["digest"][i].tobytes(), (g["labels"][i], int(g["level"][i]))


def test_inflate_malformed(tc, oracle_mod):
    g = load_golden("zlib_malformed.npz")
    streams = [unpack(g["comp"], g["comp_off"], g["comp_len"], i) for i in range(len(g["cap"]))]
    caps = [int(c) for c in g["cap"]]
    rv, outs = ragged_inflate(tc, streams, caps)
    for i, s in enumerate(streams):
        orv, oout = oracle_mod.zlib_uncompress(s, caps[i])
        assert rv[i] == orv, (i, rv[i], orv, s[:12])
        want = int(g["rv"][i])
        if want >= 0:
            assert rv[i] == want and hashlib.sha256(outs[i]).digest() == g["digest"][i].tobytes(), i
        else:
            assert rv[i] < 0


def _host_streams(oracle_mod):
    """Pages of every pagegen distribution plus skewed-random pages (long codes), encoded by the
    host zlib with every strategy and several levels."""
    rng = np.random.default_rng(7)
    pages = []
    for dist in range(6):
        for plen in (4096, 16384, 32768):
            pages.append(oracle_mod.pagegen(1, plen, seed=11, first=100 * dist + plen // 4096, dist=dist)[0].tobytes())
    for k in range(6):
        # geometric byte distribution: many rare symbols -> 11..15-bit codes
        p = 0.5 ** np.arange(1, 257) + 1e-9
        p /= p.sum()
        pages.append(rng.choice(256, size=16384, p=np.roll(p, 17 * k)).astype(np.uint8).tobytes())
    out = []
    strategies = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]
    for j, page in enumerate(pages):
        for st in strategies:
            for level in (1, 6, 9):
                if st != zlib.Z_DEFAULT_STRATEGY and level != 6:
                    continue
                c = zlib.compressobj(level, zlib.DEFLATED, 15, 8, st)
                out.append((page, c.compress(page) + c.flush()))
    return out


def test_inflate_host_zlib_strategies(tc, oracle_mod):
    pairs = _host_streams(oracle_mod)
    streams = [c for _, c in pairs]
    caps = [len(p) for p, _ in pairs]
    rv, outs = ragged_inflate(tc, streams, caps)
    for i, (page, comp) in enumerate(pairs):
        assert rv[i] == len(page), (i, rv[i])
        assert outs[i] == page, i
        assert oracle_mod.zlib_uncompress(comp, len(page))[0] == len(page)


def test_inflate_flushed_multiblock(tc):
    """Several blocks per stream (Z_FULL_FLUSH inserts empty stored blocks and byte alignment)."""
    rng = np.random.default_rng(3)
    pages, streams = [], []
    for k in range(8):
        page = bytes(rng.integers(0, 8, 12000, dtype=np.uint8)) + bytes(range(256)) * 8
        c = zlib.compressobj(6)
        s = b""
        for j in range(0, len(page), 1000 + 300 * k):
            s += c.compress(page[j:j + 1000 + 300 * k]) + c.flush(zlib.Z_FULL_FLUSH)
        s += c.flush()
        pages.append(page)
        streams.append(s)
    rv, outs = ragged_inflate(tc, streams, [len(p) for p in pages])
    for i in range(len(pages)):
        assert rv[i] == len(pages[i]) and outs[i] == pages[i], i


def test_inflate_buffer_api(tc):
    """buffer__decompress(ZLIB): Z_OK and exactly data_length bytes (src/buffer.c:257-260)."""
    from tyche_amd import buffer as B
    from tyche_amd._lib import E_OK
    g = load_golden("kat_lorem.npz")
    text, comp = g["text"].tobytes(), g["zlib"].tobytes()

    def compressed_buffer(data_length):
        buf = B.new_buffer(b"\0" * data_length, id=9)
        mem = B._libc.malloc(len(comp))
        ctypes.memmove(mem, comp, len(comp))
        B.swap_data(buf, mem)
        buf.contents.comp_length = len(comp)
        return buf

    buf = compressed_buffer(4096)
    assert B.buffer__decompress(buf, ZLIB) == E_OK
    assert buf.contents.comp_length == 0 and buf.contents.comp_hits == 1
    assert B.buffer_bytes(buf) == text
    B.destroy(buf)
    for n in (4095, 4097):          # too small: Z_BUF_ERROR; too large: Z_OK but the wrong length
        buf = compressed_buffer(n)
        assert B.buffer__decompress(buf, ZLIB) == 126
        assert buf.contents.comp_length == len(comp)
        B.destroy(buf)


def test_inflate_large_batch(tc, oracle_mod):
    """16K pages of the bench distribution: fixed-stride slots, all exact; decoding twice is identical."""
    n, plen = 16384, 16384
    host = oracle_mod.pagegen(256, plen, seed=99, first=0, dist=0)
    comps = [zlib.compress(host[i].tobytes(), 1) for i in range(256)]
    slot = (max(len(c) for c in comps) + 127) // 128 * 128
    slots = np.zeros((n, slot), np.uint8)
    clen = np.zeros(n, np.int32)
    for i in range(n):
        c = comps[i % 256]
        slots[i, :len(c)] = np.frombuffer(c, np.uint8)
        clen[i] = len(c)
    d_slots = torch.from_numpy(slots).to(DEV)
    d_clen = torch.from_numpy(clen).to(DEV)
    out, rv = tc.decompress_pages(d_slots, d_clen, plen, compressor_id=ZLIB)
    out2, rv2 = tc.decompress_pages(d_slots, d_clen, plen, compressor_id=ZLIB)
    torch.cuda.synchronize()
    assert bool((rv == plen).all())
    ref = torch.from_numpy(np.stack([host[i % 256] for i in range(n)])).to(DEV)
    assert torch.equal(out, ref) and torch.equal(out2, out) and torch.equal(rv2, rv)
