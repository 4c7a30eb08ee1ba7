"""The host side of the engine as tyche's threads see it (include/tyche_codec.h).

tyche is one process that calls the codec from opts.cpu_count compressor
threads (src/list.c:142-168, 1051) and its workers (src/list.c:572) at once,
with no notion of devices.  Covered here:

* CPU: the multi-device fan-out plan (tyche_plan_split) for any injected
  device count -- contiguous ranges, every page exactly once, balanced input
  bytes, no part below the minimum.
* GPU: 300 threads calling buffer__compress / buffer__decompress directly
  (tools/stress.c: more callers than staging contexts, far more launches than
  any fixed counter ring) with every page verified; the C5-shaped
  sweep/restore cycle (tools/cycle.c: mixed 8/16/32 KiB pages, LZ4 + zlib
  tags, a compressor pool of 250-victim batches, 64 biased restorer threads
  through the restore queue) on the GPU, and again with the fan-out rehearsed
  over four "devices" (TYCHE_DEVICE_IDS=0,0,0,0) and small fan-out parts; a
  host batch that fails part-way leaves no chunk behind for the next call.
"""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from tyche_amd import _lib

TOOLS = os.path.join(ROOT, "tools", "bin")


def _plan(lens, ndev, min_bytes):
    lib = _lib.load()
    n = len(lens)
    arr = (ctypes.c_uint32 * max(n, 1))(*lens)
    cuts = (ctypes.c_size_t * (max(ndev, 1) + 1))()
    k = lib.tyche_plan_split(n, arr, ndev, min_bytes, cuts)
    return [cuts[i] for i in range(k + 1)]


def test_plan_split_small_batches_stay_whole():
    assert _plan([], 8, 64 << 20) == [0, 0]
    assert _plan([16384] * 1000, 8, 64 << 20) == [0, 1000]          # 16 MiB < two parts' worth
    assert _plan([16384] * 1000, 1, 0) == [0, 1000]


@pytest.mark.parametrize("ndev", [2, 3, 4, 7, 8])
def test_plan_split_even_pages(ndev):
    n = 100_000
    cuts = _plan([16384] * n, ndev, 64 << 20)
    assert cuts[0] == 0 and cuts[-1] == n and len(cuts) == ndev + 1
    sizes = np.diff(cuts)
    assert (sizes > 0).all() and sizes.max() - sizes.min() <= 1


def test_plan_split_ragged_balances_bytes():
    rng = np.random.default_rng(7)
    lens = rng.choice([8192, 16384, 32768], size=50_000).astype(np.uint32)
    for ndev in (2, 5, 8):
        cuts = _plan(lens.tolist(), ndev, 1 << 20)
        assert len(cuts) == ndev + 1 and cuts[-1] == len(lens)
        part = [int(lens[a:b].sum()) for a, b in zip(cuts[:-1], cuts[1:])]
        assert sum(part) == int(lens.sum())
        assert max(part) - min(part) <= 2 * 32768                     # within a page either side of the goal


def test_plan_split_respects_minimum_part():
    # 8 devices but only ~2.5 minimum parts of input: 2 parts
    lens = [16384] * 10_000                                            # 156.25 MiB
    cuts = _plan(lens, 8, 64 << 20)
    assert len(cuts) == 3 and cuts[-1] == 10_000
    assert all(b - a >= 4096 for a, b in zip(cuts[:-1], cuts[1:]))


def _run_tool(args, env_extra=None, timeout=100, all_lines=False):
    exe = os.path.join(TOOLS, args[0])
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built")
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run([exe] + [str(a) for a in args[1:]], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=timeout, env=env)
    out = p.stdout.decode()
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert p.returncode == 0 and lines, (p.returncode, out[-2000:], p.stderr.decode()[-2000:])
    return [json.loads(l) for l in lines] if all_lines else json.loads(lines[-1])


@pytest.mark.gpu
def test_buffer_api_300_concurrent_threads():
    r = _run_tool(["stress", 300, 6])
    assert r["threads"] == 300 and r["round_trips"] == 300 * 6
    assert r["mismatches"] == 0 and r["errors"] == 0


@pytest.mark.gpu
def test_c5_cycle_one_process():
    r = _run_tool(["cycle", 12000, 64, 300, 16])
    assert r["sweep_fails"] == 0 and r["mismatches"] == 0
    assert r["restored"] > 0 and r["queue_batches"] < r["restored"]


@pytest.mark.gpu
def test_c5_live_cycle():
    """C5 as a live cycle (tools/cycle_live.c): the data set starts zlib-compressed, 64 restorers with
    the 20/80 hot-set bias restore hits through the queue while the sweeper -- raw budget 10 % of the
    data set (below the hot set, so hot pages are swept and restored again), goal overflow + 5 %, 1,000-victim flushes -- LZ4-compresses victims through a 16-thread
    compressor pool at the same time.  Both codecs restore, sweeps happen during the run, and every
    page is bit-exact at the end."""
    r = _run_tool(["cycle_live", 12000, 64, 600, 16, 10], timeout=150)
    print(r)
    assert r["mismatches"] == 0 and r["sweep_fails"] == 0, r
    assert r["restored_zlib"] > 0 and r["restored_lz4"] > 0, r    # pages swept during the run were restored again
    assert r["swept"] > 0 and r["sweeps"] > 0 and r["flushes"] >= r["sweeps"]
    assert r["queue_batches"] < r["restored"]                  # the queue coalesced concurrent restores


@pytest.mark.gpu
def test_c5_live_cycle_sustained():
    """The live cycle held for 10 s of wall time (tools/cycle_live.c seconds mode): the sweeper runs
    100+ sweeps against 64 restorers, pages cross zlib -> raw -> LZ4 -> raw many times, every page is
    bit-exact at the end, every restore went through the queue, and the histograms (compressor-pool
    call sizes, sweep flush sizes, restore launch sizes) account for every call, flush and launch."""
    r, h = _run_tool(["cycle_live", 12000, 64, 600, 16, 10, 10], timeout=200, all_lines=True)
    print(r, h)
    assert r["run_s"] >= 10.0 and r["sweeps"] >= 100, r
    assert r["mismatches"] == 0 and r["sweep_fails"] == 0, r
    assert r["restored_lz4"] > r["restored_zlib"] > 0, r      # swept pages come back again and again
    assert r["queue_buffers"] == r["restored"] and r["queue_batches"] < r["restored"], r
    assert sum(h["restore_launch_sizes"]) == r["queue_batches"], h
    assert sum(h["sweep_flush_sizes"]) == r["flushes"], h
    assert sum(h["compress_call_sizes"]) >= r["flushes"], h   # a flush is split into calls of <= 250 victims


@pytest.mark.gpu
def test_c5_live_cycle_fanout_rehearsal():
    """The live cycle with a four-entry device set (all device 0 on a one-GPU box) and 1 MiB fan-out parts."""
    r = _run_tool(["cycle_live", 8000, 64, 400, 8, 10], {"TYCHE_DEVICE_IDS": "0,0,0,0",
                                                         "TYCHE_FANOUT_MIN_BYTES": "1048576"}, timeout=150)
    assert r["devices"] == 4
    assert r["mismatches"] == 0 and r["sweep_fails"] == 0 and r["swept"] > 0 and r["restored_lz4"] > 0


@pytest.mark.gpu
def test_c5_cycle_fanout_rehearsal():
    """Four entries in the device set (all device 0 on a one-GPU box) and 1 MiB fan-out parts:
    sweep batches are split four ways and run concurrently, restores spread by load."""
    r = _run_tool(["cycle", 8000, 64, 200, 8], {"TYCHE_DEVICE_IDS": "0,0,0,0", "TYCHE_FANOUT_MIN_BYTES": "1048576"})
    assert r["devices"] == 4
    assert r["sweep_fails"] == 0 and r["mismatches"] == 0 and r["restored"] > 0


@pytest.mark.gpu
def test_failed_host_batch_leaves_nothing_for_the_next_call(oracle_mod):
    """A host batch whose second chunk cannot launch (a page capacity the decoders cannot stage)
    fails with TYCHE_E_DEVICE after its first chunk is already in flight; the staging context goes
    back to the pool drained, so the next call on the same thread gets exactly its own results."""
    lib = _lib.load()
    assert lib.tyche_set_device(0) == 0
    try:
        O = oracle_mod
        plen = 16384
        n = 12_000                                       # ~6 KB streams: two 64 MiB staging chunks
        pages = O.pagegen(n, plen, seed=99, dist=0)
        cap = O.lz4_bound(plen)
        comp = np.zeros((n, cap), dtype=np.uint8)
        clen = np.zeros(n, dtype=np.int32)
        O.lz4_compress_pages(pages, comp, clen, 0, n)
        bad_cap = 1 << 20                                # LDS for a 1 MiB page window: no decoder takes it
        out = np.zeros((n + 1, plen), dtype=np.uint8)
        big = np.zeros(bad_cap, dtype=np.uint8)
        vp = ctypes.c_void_p * (n + 1)
        src = vp(*([comp.ctypes.data + i * cap for i in range(n)] + [comp.ctypes.data]))
        slen = (ctypes.c_uint32 * (n + 1))(*([int(x) for x in clen] + [int(clen[0])]))
        dst = vp(*([out.ctypes.data + i * plen for i in range(n)] + [big.ctypes.data]))
        dcap = (ctypes.c_uint32 * (n + 1))(*([plen] * n + [bad_cap]))
        res = np.zeros(n + 1, dtype=np.int32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        rc = lib.tyche_decompress_host(1, n + 1, src, slen, dst, dcap, res.ctypes.data_as(i32p))
        assert rc == _lib.E_DEVICE, (rc, _lib.last_error())
        # the next call: a small batch with arrays sized exactly for it
        m = 100
        out2 = np.zeros((m, plen), dtype=np.uint8)
        res2 = np.full(m, -7, dtype=np.int32)
        src2 = (ctypes.c_void_p * m)(*[comp.ctypes.data + i * cap for i in range(m)])
        slen2 = (ctypes.c_uint32 * m)(*[int(x) for x in clen[:m]])
        dst2 = (ctypes.c_void_p * m)(*[out2.ctypes.data + i * plen for i in range(m)])
        dcap2 = (ctypes.c_uint32 * m)(*([plen] * m))
        rc = lib.tyche_decompress_host(1, m, src2, slen2, dst2, dcap2, res2.ctypes.data_as(i32p))
        assert rc == 0, _lib.last_error()
        assert (res2 == plen).all()
        assert np.array_equal(out2, pages[:m])
    finally:
        lib.tyche_set_device(_lib.ALL_DEVICES)


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [1, 0])
def test_host_decompress_chunks(oracle_mod, knobs, direct):
    """The host path's chunked LZ4 decompress, the kernels writing pages straight into the pinned
    arena (HOST_DIRECT_OUT=1, the default) and staged through HBM and a D2H copy (0): a ragged
    multi-chunk batch -- 8 and 16 KiB pages, every pagegen distribution, every 7th stream
    corrupted, every 11th destination short -- gives the restated LZ4_decompress_safe's result for
    every page and its bytes for every page that decodes."""
    knobs(HOST_DIRECT_OUT=direct, HOST_CHUNK_MB=8)
    lib = _lib.load()
    assert lib.tyche_set_device(0) == 0
    try:
        O = oracle_mod
        rng = np.random.default_rng(606 + direct)
        n = 6000
        plens = np.where(np.arange(n) % 3 == 0, 8192, 16384)
        pages = [O.pagegen(1, int(plens[i]), seed=5 + i, first=i, dist=i % 6)[0] for i in range(n)]
        streams, caps = [], []
        for i in range(n):
            c = bytearray(O.lz4_compress(pages[i].tobytes()))
            if i % 7 == 3:
                c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
            streams.append(bytes(c))
            caps.append(int(plens[i]) if i % 11 != 5 else int(rng.integers(100, int(plens[i]))))
        bufs = [np.frombuffer(s, dtype=np.uint8).copy() for s in streams]
        outs = [np.zeros(c, dtype=np.uint8) for c in caps]
        vp = ctypes.c_void_p * n
        src = vp(*[b.ctypes.data for b in bufs])
        slen = (ctypes.c_uint32 * n)(*[len(s) for s in streams])
        dst = vp(*[o.ctypes.data for o in outs])
        dcap = (ctypes.c_uint32 * n)(*caps)
        res = np.zeros(n, dtype=np.int32)
        rc = lib.tyche_decompress_host(1, n, src, slen, dst, dcap, res.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        assert rc == 0, _lib.last_error()
        for i in range(n):
            r, want = O.lz4_decompress(streams[i], caps[i])
            assert res[i] == r, (i, res[i], r)
            if r > 0:
                assert outs[i][:r].tobytes() == want[:r], i
    finally:
        lib.tyche_set_device(_lib.ALL_DEVICES)
