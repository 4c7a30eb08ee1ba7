"""Host-side mirror of tyche's Buffer codec interface (reference src/buffer.h:62-69).

Python wrappers over the drop-in C symbols in libtyche_codec.so, so tests and
tools can drive the exact entry points tyche's C code links against:

    buf = new_buffer(page_bytes, id=205)          # buffer__initialize(&buf, id, size, data, NULL)
    rv, comp = buffer__compress(buf, LZ4_COMPRESSOR_ID, 1)
    swap_data(buf, comp)                           # what list__update's CoW install does (list.c:1058)
    rv = buffer__decompress(buf, LZ4_COMPRESSOR_ID)

Return values are the reference's error codes (src/globals.h:35-58).
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import Buffer

_libc = ctypes.CDLL(None)
_libc.malloc.restype = ctypes.c_void_p
_libc.malloc.argtypes = [ctypes.c_size_t]
_libc.free.restype = None
_libc.free.argtypes = [ctypes.c_void_p]


def new_buffer(data: bytes | None, id: int = 0) -> ctypes.POINTER(Buffer):
    """buffer__initialize with a malloc'd copy of ``data`` (None -> blank buffer)."""
    lib = _lib.load()
    bp = ctypes.POINTER(Buffer)()
    if data is None:
        rc = lib.buffer__initialize(ctypes.byref(bp), id, 0, None, None)
    else:
        mem = _libc.malloc(max(len(data), 1))
        ctypes.memmove(mem, data, len(data))
        rc = lib.buffer__initialize(ctypes.byref(bp), id, len(data), mem, None)
    if rc != _lib.E_OK:
        raise RuntimeError(f"buffer__initialize returned {rc}")
    return bp


def buffer_bytes(bp) -> bytes:
    b = bp.contents
    n = b.comp_length if b.comp_length > 0 else b.data_length
    if not b.data or n == 0:
        return b""
    return ctypes.string_at(b.data, n)


def buffer__compress(bp, compressor_id: int, compressor_level: int = 1):
    """(rv, compressed pointer or None).  The pointer is malloc'd memory the caller owns."""
    out = ctypes.c_void_p()
    rv = _lib.load().buffer__compress(bp, ctypes.byref(out), compressor_id, compressor_level)
    return rv, (out.value if out.value else None)


def buffer__decompress(bp, compressor_id: int) -> int:
    return _lib.load().buffer__decompress(bp, compressor_id)


def swap_data(bp, new_data_ptr: int) -> None:
    """Install compressed data like the reference's tests do (tests.c:424-427): free old, point at new."""
    b = bp.contents
    if b.data:
        _libc.free(b.data)
    b.data = new_data_ptr


def destroy(bp, destroy_data: bool = True) -> None:
    _lib.load().buffer__destroy(bp, destroy_data)


def buffers_compress(bufs, compressor_id: int, compressor_level: int = 1):
    """Batch form (tyche_buffers_compress): returns (rc, statuses, compressed pointers)."""
    n = len(bufs)
    arr = (ctypes.POINTER(Buffer) * n)(*bufs)
    outs = (ctypes.c_void_p * n)()
    st = (ctypes.c_int * n)()
    rc = _lib.load().tyche_buffers_compress(arr, outs, st, n, compressor_id, compressor_level)
    return rc, list(st), [outs[i] for i in range(n)]


def buffers_decompress(bufs, compressor_id: int):
    n = len(bufs)
    arr = (ctypes.POINTER(Buffer) * n)(*bufs)
    st = (ctypes.c_int * n)()
    rc = _lib.load().tyche_buffers_decompress(arr, st, n, compressor_id)
    return rc, list(st)


def free_ptr(p: int | None) -> None:
    if p:
        _libc.free(p)
