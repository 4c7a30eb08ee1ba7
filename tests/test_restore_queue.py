"""The restore queue (§8f rank 1): concurrent per-hit restores of list__search
(src/list.c:563-589) coalesced into shared GPU batches by tyche_buffer_restore.

CPU: the queue mechanics -- every concurrent caller gets exactly the status
buffer__decompress gives it (here the no-device error), and requests coalesce
into fewer launches than callers.
GPU: 16 threads restoring LZ4 / zlib / zstd pages through the queue get their
pages back bit-exactly, with the buffer__decompress side effects.
"""
import ctypes
import threading

import numpy as np
import pytest

from tyche_amd import _lib
from tyche_amd import buffer as B


def _compressed_buffer(payload: bytes, data_length: int, id: int):
    buf = B.new_buffer(b"\0" * data_length, id=id)
    mem = B._libc.malloc(len(payload))
    ctypes.memmove(mem, payload, len(payload))
    B.swap_data(buf, mem)
    buf.contents.comp_length = len(payload)
    return buf


def _stats(lib):
    b, n = ctypes.c_uint64(), ctypes.c_uint64()
    lib.tyche_restore_queue_stats(ctypes.byref(b), ctypes.byref(n))
    return b.value, n.value


def test_queue_mechanics_cpu():
    lib = _lib.load()
    if lib.tyche_device_ready() == 1:
        pytest.skip("CPU-only mechanics test")
    bufs = [_compressed_buffer(b"\x10A", 1, i) for i in range(48)]
    direct = lib.buffer__decompress(bufs[0], 1)
    b0, n0 = _stats(lib)
    assert lib.tyche_restore_queue_start(64, 20000) == 0
    st = [None] * len(bufs)
    gate = threading.Barrier(len(bufs))

    def worker(i):
        gate.wait()
        st[i] = lib.tyche_buffer_restore(bufs[i], 1)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(bufs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    lib.tyche_restore_queue_stop()
    b1, n1 = _stats(lib)
    assert st == [direct] * len(bufs)
    assert n1 - n0 == len(bufs) and 1 <= b1 - b0 < len(bufs)
    for b in bufs:
        B.destroy(b)


@pytest.mark.gpu
def test_queue_restores_gpu(oracle_mod):
    import zlib
    lib = _lib.load()
    assert lib.tyche_device_ready() == 1, _lib.last_error()
    O = oracle_mod
    pages = O.pagegen(192, 16384, seed=44, dist=0)
    items = []
    for i in range(192):
        p = pages[i].tobytes()
        codec = (1, 2, 3)[i % 3]
        if codec == 1:
            c = O.lz4_compress(p)
        elif codec == 2:
            c = zlib.compress(p, 1)
        else:
            c = O.ref_zstd_compress(p, 1) if O.have_ref() else None
            if c is None:
                codec, c = 1, O.lz4_compress(p)
        items.append((_compressed_buffer(c, 16384, i), codec, p))
    b0, n0 = _stats(lib)
    assert lib.tyche_restore_queue_start(256, 200) == 0
    st = [None] * len(items)

    def worker(t):
        for i in range(t, len(items), 16):
            buf, codec, _ = items[i]
            st[i] = lib.tyche_buffer_restore(buf, codec)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    lib.tyche_restore_queue_stop()
    b1, n1 = _stats(lib)
    assert st == [0] * len(items)
    assert n1 - n0 == len(items) and b1 - b0 < len(items)
    for buf, codec, p in items:
        assert buf.contents.comp_length == 0 and buf.contents.comp_hits == 1
        assert B.buffer_bytes(buf) == p
        B.destroy(buf)
