"""GPU parity: the gfx950 LZ4 kernels, called through the C ABI, against the
reference's outputs (tests/golden, from vendored LZ4 1.7.5) and the oracle.

decode  -- bit-exact output and the exact LZ4_decompress_safe return value
           (lz4.c:1251; -(consumed)-1 on malformed input) for reference-encoded
           pages, the 60 sample_data pages, and corrupted/truncated streams.
encode  -- every GPU-compressed page decodes with the oracle restatement of the
           reference decoder (and with oracle/_ref, the reference build itself,
           when that .so is present) back to the input; compressed sizes stay
           within LZ4_compressBound (lz4.h:148).
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import load_golden, unpack

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def tc():
    from tyche_amd import _lib, codec
    lib = _lib.load()
    assert lib.tyche_device_ready() == 1, _lib.last_error()
    return codec


def ragged_decode(tc, streams, caps):
    """Decode a list of byte strings with per-page capacities through the general batch API."""
    n = len(streams)
    lens = [len(s) for s in streams]
    offs = np.zeros(n, np.int64)
    pos = 0
    for i, s in enumerate(streams):
        offs[i] = pos
        pos += (len(s) + 15) // 16 * 16 + 16
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
    d_offs = torch.from_numpy(offs.astype(np.uint64).view(np.int64)).to(DEV)
    d_lens = torch.tensor(lens, dtype=torch.int32, device=DEV)
    d_caps = torch.tensor(caps, dtype=torch.int32, device=DEV)
    d_ooffs = torch.from_numpy(ooffs).to(DEV)
    d_rv = torch.empty(n, dtype=torch.int32, device=DEV)
    tc.decompress_ragged(d_stream, d_offs, d_lens, d_caps, d_out, d_ooffs, d_rv,
                         max_src_length=max(lens + [1]), max_capacity=max(caps + [0]))
    torch.cuda.synchronize()
    rv = d_rv.cpu().numpy()
    out = d_out.cpu().numpy()
    return rv, [out[ooffs[i]:ooffs[i] + max(int(rv[i]), 0)].tobytes() for i in range(n)]


def test_decode_kat(tc):
    g = load_golden("kat_lorem.npz")
    rv, outs = ragged_decode(tc, [g["lz4"].tobytes()], [4096])
    assert rv[0] == 4096 and outs[0] == g["text"].tobytes()


def test_decode_reference_generated(tc, oracle_mod):
    g = load_golden("lz4_generated.npz")
    streams = [unpack(g["comp"], g["comp_off"], g["comp_len"], i) for i in range(len(g["meta"]))]
    caps = [int(m[1]) for m in g["meta"]]
    rv, outs = ragged_decode(tc, streams, caps)
    for i in range(len(streams)):
        assert rv[i] == caps[i], (i, rv[i])
        assert hashlib.sha256(outs[i]).digest() == g["digest"][i].tobytes(), i


def test_decode_reference_sample_pages(tc):
    g = load_golden("lz4_sample.npz")
    n = len(g["names"])
    streams = [unpack(g["comp"], g["comp_off"], g["comp_len"], i) for i in range(n)]
    caps = [int(s) for s in g["size"]]
    rv, outs = ragged_decode(tc, streams, caps)
    for i in range(n):
        assert rv[i] == caps[i]
        assert hashlib.sha256(outs[i]).digest() == g["digest"][i].tobytes(), g["names"][i]


def test_decode_malformed_exact_return(tc):
    g = load_golden("lz4_malformed.npz")
    n = len(g["cap"])
    streams = [unpack(g["comp"], g["comp_off"], g["comp_len"], i) for i in range(n)]
    caps = [int(c) for c in g["cap"]]
    rv, outs = ragged_decode(tc, streams, caps)
    for i in range(n):
        assert rv[i] == g["rv"][i], (i, streams[i][:12], caps[i], rv[i], g["rv"][i])
        if g["defined"][i]:
            assert hashlib.sha256(outs[i]).digest() == g["digest"][i].tobytes(), i


# device bytes / reference bytes per (page size, distribution), measured (r06_ratio_probe.jsonl);
# dist 3 is the all-zero page (~50 B per page, a few bytes of which are the excess)
LZ4_PIN = {(8192, 0): 1.0155, (8192, 1): 1.0226, (8192, 2): 0.9820, (8192, 3): 1.2326, (8192, 4): 1.0000,
           (8192, 5): 1.0114, (16384, 0): 1.0116, (16384, 1): 1.0296, (16384, 2): 0.9520, (16384, 3): 1.1067,
           (16384, 4): 1.0000, (16384, 5): 1.0084, (32768, 0): 1.0235, (32768, 1): 1.0411, (32768, 2): 0.9413,
           (32768, 3): 1.0863, (32768, 4): 1.0000, (32768, 5): 1.0114}


def ratio_bound(pins, plen, dist):
    """Allowed device/reference byte ratio: the pinned measurement + 0.5 % (1.03 or less everywhere
    but the cases the pin table shows above it)."""
    return pins[(plen, dist)] + 0.005


@pytest.mark.parametrize("dist", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("plen", [8192, 16384, 32768])
def test_encode_roundtrip_oracle(tc, oracle_mod, dist, plen):
    O = oracle_mod
    n = 48
    pages = tc.pagegen(n, plen, seed=4242, first=plen + dist * 100, dist=dist, device=DEV)
    comp, clen = tc.compress_pages(pages)
    out, rv = tc.decompress_pages(comp, clen, plen)
    torch.cuda.synchronize()
    assert torch.equal(out, pages) and bool((rv == plen).all())
    host = pages.cpu().numpy()
    ch, lh = comp.cpu().numpy(), clen.cpu().numpy()
    bound = O.lz4_bound(plen)
    ref_sizes = [len(O.lz4_compress(host[i].tobytes())) for i in range(n)]
    for i in range(n):
        assert 0 < lh[i] <= bound
        stream = ch[i, :lh[i]].tobytes()
        r, dec = O.lz4_decompress(stream, plen)
        assert r == plen and dec == host[i].tobytes()
        if O.have_ref():
            r2, dec2 = O.ref_lz4_decompress(stream, plen)
            assert r2 == plen and dec2 == host[i].tobytes()
    # ratio pinned against LZ4 1.7.5 on the same pages: the measured device/reference bytes + 0.5 %
    # (<= 1.03 but for 16/32 KiB dist 1 and the all-zero pages, where the device parse's 2^10 hash
    # slots against the reference's 2^13 cost more), so a 0.5 % ratio regression fails here
    # (tools/ratio_probe.py, profiles/r06_ratio_probe.jsonl)
    assert sum(lh) <= ratio_bound(LZ4_PIN, plen, dist) * sum(ref_sizes), (sum(lh), sum(ref_sizes))


def _literal_run_pages(n, plen, seed):
    """Pages mixing random stretches (long literal runs: batches of sequences whose encoding
    exceeds the encoder's output ring go straight to HBM, lz4_encode.hip emit_records)
    with repeated records (matches), in several proportions."""
    rng = np.random.default_rng(seed)
    pages = np.zeros((n, plen), np.uint8)
    for i in range(n):
        pos = 0
        rec = rng.integers(0, 256, 24, dtype=np.uint8)
        while pos < plen:
            kind = rng.integers(0, 4)
            m = int(rng.integers(1, [3000, 400, 60, 900][kind]))
            m = min(m, plen - pos)
            if kind in (0, 1):
                pages[i, pos:pos + m] = rng.integers(0, 256, m, dtype=np.uint8)
            else:
                pages[i, pos:pos + m] = np.resize(rec, m)
            pos += m
    return pages


@pytest.mark.parametrize("variant", ["one_wave", "split2", "split3", "split4", "split8"])
@pytest.mark.parametrize("plen", [8192, 16384, 32768])
def test_encode_kernels_long_literal_runs(tc, oracle_mod, knobs, variant, plen):
    """Every LZ4 encoder kernel (TYCHE_LZ4_ENC=1 one wave per page; the two-wave split and the
    N-wave splits, TYCHE_LZ4_ENC_WAVES, 3 being the default) on bench pages and on pages with
    long literal runs: every stream restores through the reference decoder (oracle/_ref) and
    the oracle's."""
    O = oracle_mod
    if variant == "one_wave":
        knobs(LZ4_ENC=1)
    else:
        knobs(LZ4_ENC_WAVES=int(variant[-1]))
    n = 24
    host = np.concatenate([_literal_run_pages(n, plen, plen + 7),
                           tc.pagegen(n, plen, seed=77, first=plen, dist=0, device=DEV).cpu().numpy()])
    pages = torch.from_numpy(host).to(DEV)
    comp, clen = tc.compress_pages(pages)
    torch.cuda.synchronize()
    ch, lh = comp.cpu().numpy(), clen.cpu().numpy()
    for i in range(2 * n):
        assert 0 < lh[i] <= O.lz4_bound(plen), (i, lh[i])
        stream = ch[i, :lh[i]].tobytes()
        r, dec = O.lz4_decompress(stream, plen)
        assert r == plen and dec == host[i].tobytes(), i
        if O.have_ref():
            r2, dec2 = O.ref_lz4_decompress(stream, plen)
            assert r2 == plen and dec2 == host[i].tobytes(), i
    out, rv = tc.decompress_pages(comp, clen, plen)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)


def test_pagegen_matches_host(tc, oracle_mod):
    for dist in range(6):
        d = tc.pagegen(8, 16384, seed=11, first=123, dist=dist, device=DEV).cpu().numpy()
        h = oracle_mod.pagegen(8, 16384, seed=11, first=123, dist=dist)
        assert np.array_equal(d, h), dist


@pytest.mark.parametrize("kernel", ["default", "split3_all_sizes"])
@pytest.mark.parametrize("n", [0, 1, 4, 12, 13, 14, 63, 64, 65, 100, 1000, 4095, 65535])
def test_encode_sizes(tc, oracle_mod, knobs, n, kernel):
    """Edge sizes: empty (LZ4 emits one 0x00 token), below MFLIMIT+1, around a wave, max byU16 size;
    each also through the three-wave split kernel (TYCHE_LZ4_SPLIT_MIN=0: parts of a tiny page are
    empty or a few bytes)."""
    O = oracle_mod
    if kernel != "default":
        knobs(LZ4_SPLIT_MIN=0)
    rng = np.random.default_rng(n)
    data = (rng.integers(0, 3, n, dtype=np.uint8) * 40).tobytes()
    src = torch.from_numpy(np.frombuffer(data, np.uint8).copy().reshape(1, n) if n else np.zeros((1, 0), np.uint8))
    src = src.to(DEV)
    slot = tc.slot_size(max(n, 1))
    comp = torch.zeros((1, slot), dtype=torch.uint8, device=DEV)
    clen = torch.zeros(1, dtype=torch.int32, device=DEV)
    if n == 0:
        from tyche_amd import _lib
        import ctypes
        b = _lib.Batch(count=1, src=src.data_ptr() if src.numel() else comp.data_ptr(), src_stride=0, src_length=0,
                       max_src_length=0, dst=comp.data_ptr(), dst_stride=slot, dst_capacity=slot,
                       results=clen.data_ptr())
        _lib.check(_lib.load().tyche_compress_batch(1, 1, ctypes.byref(b), torch.cuda.current_stream().cuda_stream),
                   "compress")
    else:
        tc.compress_pages(src, out=comp, out_len=clen)
    torch.cuda.synchronize()
    L = int(clen[0])
    stream = comp[0, :L].cpu().numpy().tobytes()
    if n == 0:
        assert stream == b"\x00"
    r, dec = O.lz4_decompress(stream, n)
    assert r == n and dec == data
    if n:
        out, rv = tc.decompress_pages(comp, clen, n)
        torch.cuda.synchronize()
        assert int(rv[0]) == n and out[0].cpu().numpy().tobytes() == data


def test_large_batch_properties(tc):
    """A 64K-page batch: round trip, and a checksum of checksums stable across two runs."""
    n, plen = 65536, 16384
    pages = tc.pagegen(n, plen, seed=5, dist=0, device=DEV)
    comp, clen = tc.compress_pages(pages)
    out, rv = tc.decompress_pages(comp, clen, plen)
    comp2, clen2 = tc.compress_pages(pages)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)
    assert torch.equal(clen, clen2)
    mask = torch.arange(comp.shape[1], device=DEV)[None, :] < clen[:, None].long()
    assert torch.equal(comp * mask, comp2 * mask)   # deterministic encoder


def test_too_large_reported(tc):
    """A page whose length exceeds the launch's declared maximum is refused per page, never overrun."""
    from tyche_amd import _lib
    rv, _ = ragged_decode(tc, [b"\x00" * 10], [64])
    assert rv[0] < 0


def test_buffer_api_kat(tc):
    """src/tests.c Test 4 through the drop-in buffer__compress / buffer__decompress."""
    from tyche_amd import buffer as B
    from tyche_amd._lib import LZ4_COMPRESSOR_ID, E_OK
    g = load_golden("kat_lorem.npz")
    text = g["text"].tobytes()
    buf = B.new_buffer(text, id=205)
    rv, comp = B.buffer__compress(buf, LZ4_COMPRESSOR_ID, 1)
    assert rv == E_OK and comp
    assert 0 < buf.contents.comp_length <= 4096 + 4096 // 255 + 16
    B.swap_data(buf, comp)
    assert B.buffer__decompress(buf, LZ4_COMPRESSOR_ID) == E_OK
    assert buf.contents.comp_length == 0 and buf.contents.comp_hits == 1
    assert B.buffer_bytes(buf) == text
    assert B.buffer__decompress(buf, LZ4_COMPRESSOR_ID) == 125   # already decompressed
    B.destroy(buf)


def test_buffer_batch_api(tc, oracle_mod):
    from tyche_amd import buffer as B
    pages = oracle_mod.pagegen(40, 8192, seed=3, dist=0)
    bufs = [B.new_buffer(pages[i].tobytes(), id=i) for i in range(40)]
    rc, st, ptrs = B.buffers_compress(bufs, 1, 1)
    assert rc == 0 and st == [0] * 40
    for b, p in zip(bufs, ptrs):
        B.swap_data(b, p)
    rc, st = B.buffers_decompress(bufs, 1)
    assert rc == 0 and st == [0] * 40
    for i, b in enumerate(bufs):
        assert B.buffer_bytes(b) == pages[i].tobytes()
        B.destroy(b)


def _seq_stream(nseq, tail):
    body = bytes([0x10, 0x41, 0x01, 0x00])                     # 1 literal 'A', match 4 at offset 1
    body += bytes([0x00, 0x01, 0x00]) * (nseq - 1)             # matches of 4 at offset 1
    return body + bytes([0x50]) + b"B" * 5 if tail else body   # 5 trailing literals (or none)


@pytest.mark.parametrize("nseq,cap,tail", [(6000, 16384, True), (6000, 8192, True), (3000, 16384, True),
                                           (20000, 65535, True), (4094, 16384, True), (4094, 16384, False),
                                           (2000, 8192, True)])
def test_decode_token_list_near_output(tc, oracle_mod, nseq, cap, tail):
    """Streams of thousands of 3-byte sequences (4 output bytes each): the token positions kept at the
    top of the page window would be reached by the output of a stream whose sequences overrun the
    capacity, so such pages restart on the sequential decoder.  Verdict and output equal the
    oracle's either way; (4094, 16384) exactly fills the page."""
    s = _seq_stream(nseq, tail)
    r, dec = oracle_mod.lz4_decompress(s, cap)
    rv, outs = ragged_decode(tc, [s], [cap])
    assert rv[0] == r, (rv[0], r)
    if r > 0:
        assert outs[0] == dec


def test_decode_size_classes(tc):
    """A 16K-page batch whose streams span 2 KB .. 16 KB (compressible, half-random, random pages in
    a seeded shuffle): the launch splits into a short-stream class sized for one more wave per CU
    and a long-stream class; every page is decoded exactly once, in either."""
    n, plen = 16384, 16384
    pages = tc.pagegen(n, plen, seed=17, dist=0, device=DEV)
    g = torch.Generator(device="cpu").manual_seed(3)
    noisy = torch.randperm(n, generator=g)[: n // 8].to(DEV)
    rnd = torch.randint(0, 256, (noisy.numel(), plen), dtype=torch.uint8, generator=None, device=DEV)
    half = torch.arange(noisy.numel(), device=DEV) % 2 == 0
    pages[noisy[half]] = rnd[half]                       # incompressible: streams > page
    pages[noisy[~half], : plen // 3] = rnd[~half][:, : plen // 3]   # a third random: mid-size streams
    comp, clen = tc.compress_pages(pages)
    mx = int(clen.max())
    assert mx > 16384 and int(clen.min()) < 7000
    out, rv = tc.decompress_pages(comp, clen, plen, max_comp_len=mx)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)


@pytest.mark.parametrize("target", [1, 20000, 65536])
def test_decode_lane_path_fixtures(tc, target):
    """The decoder is picked by batch size: below 16,384 pages the jump decoder (workgroup per
    page, pointer-jumping match resolution), below 32,768 the wave decoder, from there the
    lane-per-page decoder (lz4_decode_lane.hip).  The reference-generated, sample and malformed
    fixtures, repeated to each size, give the reference's return values and bytes on all three."""
    gm, gg, gs = load_golden("lz4_malformed.npz"), load_golden("lz4_generated.npz"), load_golden("lz4_sample.npz")
    streams, caps, want_rv, want_dig = [], [], [], []
    for i in range(len(gm["cap"])):
        streams.append(unpack(gm["comp"], gm["comp_off"], gm["comp_len"], i))
        caps.append(int(gm["cap"][i]))
        want_rv.append(int(gm["rv"][i]))
        want_dig.append(gm["digest"][i].tobytes() if gm["defined"][i] else None)
    for g, capf in ((gg, lambda i: int(gg["meta"][i][1])), (gs, lambda i: int(gs["size"][i]))):
        m = len(g["digest"])
        for i in range(m):
            streams.append(unpack(g["comp"], g["comp_off"], g["comp_len"], i))
            caps.append(capf(i))
            want_rv.append(caps[-1])
            want_dig.append(g["digest"][i].tobytes())
    k = -(-target // len(streams))
    rv, outs = ragged_decode(tc, streams * k, caps * k)
    for j in range(len(streams) * k):
        i = j % len(streams)
        assert rv[j] == want_rv[i], (j, i, rv[j], want_rv[i])
        if want_dig[i] is not None:
            assert hashlib.sha256(outs[j]).digest() == want_dig[i], (j, i)


@pytest.mark.parametrize("ring", [128, 160, 192, 256])
def test_decode_lc_kernel_variants(tc, oracle_mod, knobs, ring):
    """The chunked lane-per-page decoder (lz4_decode_lc.hip) at every ring size, forced on every
    batch size (LZ4_LC=1, LZ4_LANE_MIN=0): the fixtures with their exact return values, seeded
    corruptions against the restated LZ4_decompress_safe, and the page kinds that exercise its
    split records (incompressible pages: literal runs longer than a window; zero and short-period
    pages: long self-overlapping matches; deep match chains)."""
    knobs(LZ4_LC=1, LZ4_LC_RING=ring, LZ4_LANE_MIN=0)
    test_decode_lane_path_fixtures(tc, 1)
    rng = np.random.default_rng(3000 + ring)
    pages = oracle_mod.pagegen(256, 16384, seed=13, first=ring, dist=0)
    streams, caps = [], []
    for i in range(256):
        c = bytearray(oracle_mod.lz4_compress(pages[i].tobytes()))
        if i % 4 == 1:
            c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
        elif i % 4 == 2:
            c = c[: int(rng.integers(1, len(c)))]
        streams.append(bytes(c))
        caps.append(16384 if i % 4 != 3 else int(rng.integers(100, 16384)))
    rv, outs = ragged_decode(tc, streams, caps)
    for i in range(256):
        r, want = oracle_mod.lz4_decompress(streams[i], caps[i])
        assert rv[i] == r, (i, rv[i], r)
        if r > 0 and i % 4 in (0, 3):
            assert outs[i][:r] == want[:r], i
    for plen in (8192, 16384, 32768):
        test_decode_jump_path_page_kinds(tc, oracle_mod, plen, 300)
    test_decode_token_list_near_output(tc, oracle_mod, 6000, 16384, True)
    test_decode_token_list_near_output(tc, oracle_mod, 20000, 65535, True)


@pytest.mark.parametrize("dist", [0, 1, 2, 3, 4, 5])
def test_decode_lane_path_roundtrip(tc, dist):
    """64K x 4 KiB pages of every pagegen distribution through the lane-per-page decoder."""
    n, plen = 65536, 4096
    pages = tc.pagegen(n, plen, seed=77, first=dist * 1000, dist=dist, device=DEV)
    comp, clen = tc.compress_pages(pages)
    out, rv = tc.decompress_pages(comp, clen, plen)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)


@pytest.mark.parametrize("n", [600, 20000, 65536])
def test_decode_lane_path_corruptions(tc, oracle_mod, n):
    """Seeded corruptions (byte flips, truncations) through the jump (600 pages), wave
    (20,000) and lane-per-page (64K) decoders: every return value is the restated
    LZ4_decompress_safe's (lz4.c:1251), and the untouched pages decode bit-exactly."""
    plen = 4096
    pages = tc.pagegen(n, plen, seed=99, dist=0, device=DEV)
    comp, clen = tc.compress_pages(pages)
    torch.cuda.synchronize()
    ch, lh = comp.cpu().numpy().copy(), clen.cpu().numpy().astype(np.int64).copy()
    rng = np.random.default_rng(20170303)
    kind = rng.integers(0, 4, n)          # 0 clean, 1 flip, 2 truncate, 3 flip + truncate
    for i in np.nonzero(kind & 1)[0]:
        for _ in range(int(rng.integers(1, 4))):
            ch[i, rng.integers(0, lh[i])] ^= np.uint8(rng.integers(1, 256))
    for i in np.nonzero(kind & 2)[0]:
        lh[i] = int(rng.integers(0, lh[i]))
    d_comp = torch.from_numpy(ch).to(DEV)
    d_len = torch.from_numpy(lh.astype(np.int32)).to(DEV)
    out, rv = tc.decompress_pages(d_comp, d_len, plen, max_comp_len=int(ch.shape[1]))
    torch.cuda.synchronize()
    rv, out = rv.cpu().numpy(), out.cpu().numpy()
    host = pages.cpu().numpy()
    for i in range(n):
        r, dec = oracle_mod.lz4_decompress(ch[i, :lh[i]].tobytes(), plen)
        assert rv[i] == r, (i, kind[i], rv[i], r)
        if kind[i] == 0:
            assert r == plen and out[i].tobytes() == host[i].tobytes(), i


@pytest.mark.parametrize("plen", [8192, 32768, 65535])
def test_decode_lane_path_page_sizes(tc, oracle_mod, plen):
    """32K-page batches (the lane decoder's threshold) of 8 KiB (C4's page size), 32 KiB and
    65,535-byte pages: round trip on the GPU, and every page's device stream decodes identically
    with the oracle restatement (oracle_lz4_decompress_pages)."""
    n = 32768
    gen = (plen + 4095) // 4096 * 4096          # pagegen sizes; 65,535 = the byU16 limit, cut from 64 KiB
    pages = tc.pagegen(n, gen, seed=31, first=plen, dist=0, device=DEV)[:, :plen].contiguous()
    comp, clen = tc.compress_pages(pages)
    out, rv = tc.decompress_pages(comp, clen, plen)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()) and torch.equal(out, pages)
    # every page's device stream through the C oracle (LZ4_decompress_safe restated) back to the page
    ch, lh, host = comp.cpu().numpy(), clen.cpu().numpy().astype(np.int32), pages.cpu().numpy()
    dec = np.zeros_like(host)
    orv = np.zeros(n, np.int32)
    oracle_mod.lz4_decompress_pages(ch, lh, dec, orv, 0, n)
    assert bool((orv == plen).all()), np.nonzero(orv != plen)[0][:10]
    assert np.array_equal(dec, host)


@pytest.mark.parametrize("plen", [8192, 16384, 32768])
@pytest.mark.parametrize("n", [1, 7, 300])
def test_decode_jump_path_page_kinds(tc, oracle_mod, plen, n):
    """Small batches (the jump decoder) of every pagegen distribution plus pages built for its
    corner cases: incompressible (literal runs longer than a lane fills), all-zero and
    short-period pages (long self-overlapping matches, the workgroup's run list), and pages whose
    matches copy earlier matches hundreds of times (deep pointer chains).  Round trip on the GPU;
    a sample decodes identically with the oracle restatement."""
    g = torch.Generator(device="cpu").manual_seed(plen + n)
    pages = tc.pagegen(n, plen, seed=plen * 3 + n, first=n, dist=0, device=DEV)
    for i in range(n):
        kind = i % 6
        if kind == 1:
            pages[i] = torch.randint(0, 256, (plen,), dtype=torch.uint8, generator=g).to(DEV)
        elif kind == 2:
            pages[i] = 0
        elif kind == 3:
            per = int(torch.randint(1, 40, (1,), generator=g))
            pat = torch.randint(0, 256, (per,), dtype=torch.uint8, generator=g)
            pages[i] = pat.repeat(plen // per + 1)[:plen].to(DEV)
        elif kind == 4:
            src = tc.pagegen(1, plen, seed=i, first=i, dist=i % 6, device=DEV)
            pages[i] = src[0]
        elif kind == 5:
            rec = torch.randint(0, 256, (24,), dtype=torch.uint8, generator=g)
            page = rec.repeat(plen // 24 + 1)[:plen].clone()
            noise = torch.randint(0, plen, (plen // 97,), generator=g)
            page[noise] = torch.randint(0, 256, (noise.numel(),), dtype=torch.uint8, generator=g)
            pages[i] = page.to(DEV)
    comp, clen = tc.compress_pages(pages)
    mx = int(clen.max())
    out, rv = tc.decompress_pages(comp, clen, plen, max_comp_len=mx)
    torch.cuda.synchronize()
    assert bool((rv == plen).all()), rv
    assert torch.equal(out, pages)
    ch, lh, host = comp[:12].cpu().numpy(), clen[:12].cpu().numpy(), pages[:12].cpu().numpy()
    for i in range(min(n, 12)):
        r, dec = oracle_mod.lz4_decompress(ch[i, :lh[i]].tobytes(), plen)
        assert r == plen and dec == host[i].tobytes(), i


def short_sequence_stream(rng, plen):
    """A valid LZ4 block made almost entirely of 3-byte sequences (no literals, 4..18-byte matches
    at random offsets): the token chain runs in phase with period 3 for the whole page, the case
    that defeats token walks started at fixed segment offsets."""
    first = 24
    s = bytearray([0xF0 | 0, first - 15]) + bytearray(rng.integers(0, 256, first, dtype=np.uint8).tobytes())
    s += int(rng.integers(1, first + 1)).to_bytes(2, "little")
    out = first + 4
    while out < plen - 40:
        code = int(rng.integers(0, 15))
        s.append(code)
        s += int(rng.integers(1, min(out, 65535) + 1)).to_bytes(2, "little")
        out += code + 4
    lit = plen - out
    ext = lit - 15
    s.append(0xF0)
    while ext >= 255:
        s.append(255)
        ext -= 255
    s.append(ext)
    s += bytearray(rng.integers(0, 256, lit, dtype=np.uint8).tobytes())
    return bytes(s)


@pytest.mark.parametrize("kernel", ["solo", "solo_lockstep", "jump"])
def test_decode_small_batch_kernels(tc, oracle_mod, knobs, kernel):
    """The small-batch LZ4 decoders side by side: the single-page decoder (round 5, the default
    for batches of <= 4,096 pages), the same with its jump rounds handed to the lock-step loop
    after one barrier-free round (LZ4_SOLO_ASYNC=1), and the jump decoder (LZ4_SOLO_MAX=0).  The reference fixtures
    with their exact return values at 1 and 20 pages, seeded corruptions (bit flips, truncations,
    reduced capacities) against the restated LZ4_decompress_safe, crafted pages of back-to-back
    3-byte sequences (with and without corruptions), and every page kind at 8, 16 and 32 KiB."""
    if kernel == "jump":
        knobs(LZ4_SOLO_MAX=0)
    elif kernel == "solo_lockstep":
        knobs(LZ4_SOLO_ASYNC=1)
    test_decode_lane_path_fixtures(tc, 1)
    test_decode_lane_path_fixtures(tc, 20)
    rng = np.random.default_rng(4000 + len(kernel))
    pages = oracle_mod.pagegen(300, 16384, seed=17, first=len(kernel), dist=0)
    streams, caps = [], []
    for i in range(300):
        c = bytearray(oracle_mod.lz4_compress(pages[i].tobytes()))
        if i % 4 == 1:
            c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
        elif i % 4 == 2:
            c = c[: int(rng.integers(1, len(c)))]
        streams.append(bytes(c))
        caps.append(16384 if i % 4 != 3 else int(rng.integers(100, 16384)))
    rv, outs = ragged_decode(tc, streams, caps)
    for i in range(300):
        r, want = oracle_mod.lz4_decompress(streams[i], caps[i])
        assert rv[i] == r, (i, rv[i], r)
        if r > 0 and i % 4 in (0, 3):
            assert outs[i][:r] == want[:r], i
    streams = [short_sequence_stream(rng, 16384) for _ in range(24)]
    for i in range(8, 24, 2):
        c = bytearray(streams[i])
        c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
        streams[i] = bytes(c)
    for n in (1, 24):
        rv, outs = ragged_decode(tc, streams[:n], [16384] * n)
        for i in range(n):
            r, want = oracle_mod.lz4_decompress(streams[i], 16384)
            assert rv[i] == r, (i, rv[i], r)
            assert r < 0 or outs[i][:r] == want[:r], i
    for plen in (8192, 16384, 32768):
        test_decode_jump_path_page_kinds(tc, oracle_mod, plen, 7)
        test_decode_jump_path_page_kinds(tc, oracle_mod, plen, 300)


def test_c2_full_size_round_trip(tc):
    """BASELINE configs[1] at its full size on one GPU: 1,048,576 x 16 KiB synthetic pages
    (16 GiB) LZ4-compressed and decompressed through the lane decoder, every page bit-exact,
    every result the page length, and the ratio of the bench pages (the bench checks the same
    round trip; this keeps it in the parity suite)."""
    n, plen = 1 << 20, 16384
    pages = tc.pagegen(n, plen, dist=0, device=DEV)
    comp, clen = tc.compress_pages(pages)
    out, rv = tc.decompress_pages(comp, clen, plen)
    torch.cuda.synchronize()
    assert bool((rv == plen).all())
    assert torch.equal(out, pages)
    ratio = n * plen / float(clen.to(torch.int64).sum())
    # pinned: the bench pages' ratio is 2.6175 (r05/r06 bench lines; LZ4 1.7.5 gets 2.647)
    assert 2.61 <= ratio < 2.7, ratio
    del pages, comp, out
    torch.cuda.empty_cache()


def test_scratch_oom_recovered(tc, knobs, oracle_mod):
    """A scratch lease whose first hipMalloc fails (SCRATCH_OOM_SEQ: an oversized real request, so
    the HIP error slot is set exactly as by an out-of-memory) frees the idle pool, retries and
    succeeds; the launch that follows must not report the recovered failure (engine.hip
    ScratchLease: the error slot is cleared), and the split encoder's output still round-trips."""
    n, plen = 2048, 16384
    pages = tc.pagegen(n, plen, dist=0, device=DEV)
    for seq in (1, 2):   # each new value forces one failure
        knobs(SCRATCH_OOM_SEQ=seq)
        comp, clen = tc.compress_pages(pages)   # raises on a non-zero engine status
        out, rv = tc.decompress_pages(comp, clen, plen)
        torch.cuda.synchronize()
        assert bool((clen > 0).all()) and bool((rv == plen).all())
        assert torch.equal(out, pages)
    ch, lh = comp[:4].cpu().numpy(), clen[:4].cpu().numpy()
    host = pages[:4].cpu().numpy()
    for i in range(4):
        r, dec = oracle_mod.lz4_decompress(ch[i, :lh[i]].tobytes(), plen)
        assert r == plen and dec == host[i].tobytes()
