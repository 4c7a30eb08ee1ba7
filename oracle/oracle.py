"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU checkers built by oracle/Makefile:

* ``liboracle.so``: this repo's clean-room restatement of LZ4 1.7.5
  (oracle/lz4_oracle.c) plus the host copy of the synthetic page generator.
* ``_ref/libtyche_ref.so``: the reference's vendored codecs compiled from
  /root/reference/src (only present where that tree was available at build time;
  the .so travels to the GPU box with the snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (tyche_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libtyche_ref.so")
REF_TREE = "/root/reference/src"

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)


def build(ref: bool | None = None) -> None:
    """Compile liboracle.so (and _ref when the reference tree exists)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    if ref is None:
        ref = os.path.isdir(REF_TREE)
    if ref:
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


class _Lib:
    _oracle = None
    _ref = None

    @classmethod
    def oracle(cls):
        if cls._oracle is None:
            if not os.path.exists(ORACLE_SO):
                build(ref=False)
            lib = ctypes.CDLL(ORACLE_SO)
            for name in ("oracle_lz4_compress", "oracle_lz4_compress_default", "oracle_lz4_decompress_safe"):
                f = getattr(lib, name)
                f.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int]
                f.restype = ctypes.c_int
            lib.oracle_lz4_compress_bound.argtypes = [ctypes.c_int]
            lib.oracle_lz4_compress_bound.restype = ctypes.c_int
            lib.oracle_lz4_compress_pages.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, _u8p, ctypes.c_uint64,
                                                      _i32p, ctypes.c_long, ctypes.c_long]
            lib.oracle_lz4_compress_pages.restype = ctypes.c_long
            lib.oracle_lz4_decompress_pages.argtypes = [_u8p, ctypes.c_uint64, _i32p, _u8p, ctypes.c_uint64,
                                                        ctypes.c_uint32, _i32p, ctypes.c_long, ctypes.c_long]
            lib.oracle_lz4_decompress_pages.restype = ctypes.c_long
            lib.oracle_pagegen.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_long, ctypes.c_uint32]
            lib.oracle_pagegen.restype = None
            lib.oracle_zlib_uncompress.argtypes = [_u8p, ctypes.c_int, _u8p, ctypes.c_int]
            lib.oracle_zlib_uncompress.restype = ctypes.c_int
            lib.oracle_adler32.argtypes = [_u8p, ctypes.c_int]
            lib.oracle_adler32.restype = ctypes.c_uint32
            lib.oracle_zstd_decompress.argtypes = [_u8p, ctypes.c_int, _u8p, ctypes.c_int]
            lib.oracle_zstd_decompress.restype = ctypes.c_int
            lib.oracle_zstd_compress_bound.argtypes = [ctypes.c_int]
            lib.oracle_zstd_compress_bound.restype = ctypes.c_int
            lib.oracle_xxh64.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint64]
            lib.oracle_xxh64.restype = ctypes.c_uint64
            cls._oracle = lib
        return cls._oracle

    @classmethod
    def ref(cls):
        if cls._ref is None:
            if not os.path.exists(REF_SO):
                return None
            lib = ctypes.CDLL(REF_SO)
            lib.LZ4_compress_default.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int]
            lib.LZ4_compress_default.restype = ctypes.c_int
            lib.LZ4_decompress_safe.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int]
            lib.LZ4_decompress_safe.restype = ctypes.c_int
            lib.LZ4_compressBound.argtypes = [ctypes.c_int]
            lib.LZ4_compressBound.restype = ctypes.c_int
            lib.compress2.argtypes = [_u8p, ctypes.POINTER(ctypes.c_ulong), _u8p, ctypes.c_ulong, ctypes.c_int]
            lib.compress2.restype = ctypes.c_int
            lib.compressBound.argtypes = [ctypes.c_ulong]
            lib.compressBound.restype = ctypes.c_ulong
            lib.uncompress.argtypes = [_u8p, ctypes.POINTER(ctypes.c_ulong), _u8p, ctypes.c_ulong]
            lib.uncompress.restype = ctypes.c_int
            lib.ZSTD_compress.argtypes = [_u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t, ctypes.c_int]
            lib.ZSTD_compress.restype = ctypes.c_size_t
            lib.ZSTD_decompress.argtypes = [_u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t]
            lib.ZSTD_decompress.restype = ctypes.c_size_t
            lib.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
            lib.ZSTD_compressBound.restype = ctypes.c_size_t
            lib.ZSTD_isError.argtypes = [ctypes.c_size_t]
            lib.ZSTD_isError.restype = ctypes.c_uint
            lib.ZSTD_createCCtx.argtypes = []
            lib.ZSTD_createCCtx.restype = ctypes.c_void_p
            lib.ZSTD_freeCCtx.argtypes = [ctypes.c_void_p]
            lib.ZSTD_freeCCtx.restype = ctypes.c_size_t
            lib.ZSTD_compressBegin.argtypes = [ctypes.c_void_p, ctypes.c_int]
            lib.ZSTD_compressBegin.restype = ctypes.c_size_t
            for name in ("ZSTD_compressContinue", "ZSTD_compressEnd"):
                f = getattr(lib, name)
                f.argtypes = [ctypes.c_void_p, _u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t]
                f.restype = ctypes.c_size_t
            lib.ZSTD_XXH64.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_ulonglong]
            lib.ZSTD_XXH64.restype = ctypes.c_ulonglong
            cls._ref = lib
        return cls._ref


def have_ref() -> bool:
    return _Lib.ref() is not None


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8)
    return np.frombuffer(bytes(data), dtype=np.uint8).copy()


# ---------------------------------------------------------------- restatement
def lz4_bound(n: int) -> int:
    return _Lib.oracle().oracle_lz4_compress_bound(n)


def lz4_compress(data, cap: int | None = None) -> bytes:
    """LZ4_compress_default restated (lz4.c:697); returns b'' when the codec returns 0."""
    src = _as_u8(data)
    n = src.size
    if cap is None:
        cap = lz4_bound(n)
    dst = np.zeros(max(cap, 1) + 64, dtype=np.uint8)
    r = _Lib.oracle().oracle_lz4_compress_default(_ptr(src), _ptr(dst), n, cap)
    return dst[:r].tobytes() if r > 0 else b""


def lz4_decompress(comp, out_cap: int) -> tuple[int, bytes]:
    """LZ4_decompress_safe restated (lz4.c:1251): (return value, decoded bytes)."""
    src = _as_u8(comp)
    if src.size == 0:
        src = np.zeros(1, dtype=np.uint8)[:0]
    dst = np.zeros(max(out_cap, 1), dtype=np.uint8)
    srcbuf = np.zeros(src.size + 16, dtype=np.uint8)
    srcbuf[:src.size] = src
    r = _Lib.oracle().oracle_lz4_decompress_safe(_ptr(srcbuf), _ptr(dst), src.size, out_cap)
    return r, (dst[:r].tobytes() if r > 0 else b"")


def zlib_uncompress(comp, out_cap: int) -> tuple[int, bytes]:
    """uncompress() restated (src/zlib/uncompr.c:22): (decoded length or negative zlib code, bytes)."""
    src = _as_u8(comp)
    srcbuf = np.zeros(src.size + 16, dtype=np.uint8)
    srcbuf[:src.size] = src
    dst = np.zeros(max(out_cap, 1), dtype=np.uint8)
    r = _Lib.oracle().oracle_zlib_uncompress(_ptr(srcbuf), src.size, _ptr(dst), out_cap)
    return r, (dst[:r].tobytes() if r > 0 else b"")


def zstd_decompress(comp, out_cap: int) -> tuple[int, bytes]:
    """ZSTD_decompress restated (zstd_decompress.c:1459): (decoded size or negative error, bytes)."""
    src = _as_u8(comp)
    srcbuf = np.zeros(src.size + 16, dtype=np.uint8)
    srcbuf[:src.size] = src
    dst = np.zeros(max(out_cap, 1) + 16, dtype=np.uint8)
    r = _Lib.oracle().oracle_zstd_decompress(_ptr(srcbuf), src.size, _ptr(dst), out_cap)
    return r, (dst[:r].tobytes() if r > 0 else b"")


def zstd_bound(n: int) -> int:
    return _Lib.oracle().oracle_zstd_compress_bound(n)


def xxh64(data, seed: int = 0) -> int:
    src = _as_u8(data)
    return int(_Lib.oracle().oracle_xxh64(_ptr(src), src.size, seed))


def adler32(data) -> int:
    src = _as_u8(data)
    return int(_Lib.oracle().oracle_adler32(_ptr(src), src.size))


def pagegen(n: int, page_len: int, seed: int = 20170303, first: int = 0, dist: int = 0) -> np.ndarray:
    """Host copy of tyche_amd/csrc/pagegen.h: (n, page_len) uint8 pages."""
    out = np.zeros((n, page_len), dtype=np.uint8)
    _Lib.oracle().oracle_pagegen(_ptr(out), page_len, page_len, seed, first, n, dist)
    return out


def lz4_compress_pages(pages: np.ndarray, dst: np.ndarray, out_len: np.ndarray, first: int, count: int) -> int:
    n, plen = pages.shape
    return _Lib.oracle().oracle_lz4_compress_pages(_ptr(pages), plen, plen, _ptr(dst), dst.shape[1],
                                                   out_len.ctypes.data_as(_i32p), first, count)


def lz4_decompress_pages(comp: np.ndarray, comp_len: np.ndarray, out: np.ndarray, rv: np.ndarray,
                         first: int, count: int) -> int:
    return _Lib.oracle().oracle_lz4_decompress_pages(_ptr(comp), comp.shape[1], comp_len.ctypes.data_as(_i32p),
                                                     _ptr(out), out.shape[1], out.shape[1],
                                                     rv.ctypes.data_as(_i32p), first, count)


# ------------------------------------------------------------ reference build
def ref_lz4_compress(data) -> bytes:
    lib = _Lib.ref()
    src = _as_u8(data)
    cap = lib.LZ4_compressBound(src.size)
    dst = np.zeros(cap + 64, dtype=np.uint8)
    r = lib.LZ4_compress_default(_ptr(src), _ptr(dst), src.size, cap)
    return dst[:r].tobytes() if r > 0 else b""


def ref_lz4_decompress(comp, out_cap: int, fill: int = 0) -> tuple[int, bytes]:
    lib = _Lib.ref()
    src = _as_u8(comp)
    srcbuf = np.zeros(src.size + 16, dtype=np.uint8)
    srcbuf[:src.size] = src
    dst = np.full(max(out_cap, 1) + 16, fill, dtype=np.uint8)
    r = lib.LZ4_decompress_safe(_ptr(srcbuf), _ptr(dst), src.size, out_cap)
    return r, (dst[:r].tobytes() if r > 0 else b"")


def ref_zlib_compress(data, level: int = 1) -> bytes:
    lib = _Lib.ref()
    src = _as_u8(data)
    cap = ctypes.c_ulong(lib.compressBound(src.size))
    dst = np.zeros(cap.value + 16, dtype=np.uint8)
    r = lib.compress2(_ptr(dst), ctypes.byref(cap), _ptr(src), src.size, level)
    assert r == 0, r
    return dst[:cap.value].tobytes()


def ref_zlib_uncompress(comp, out_cap: int) -> tuple[int, bytes]:
    """The reference's uncompress(): (decoded length or negative zlib code, bytes)."""
    lib = _Lib.ref()
    src = _as_u8(comp)
    srcbuf = np.zeros(src.size + 16, dtype=np.uint8)
    srcbuf[:src.size] = src
    dst = np.zeros(max(out_cap, 1) + 16, dtype=np.uint8)
    n = ctypes.c_ulong(out_cap)
    r = lib.uncompress(_ptr(dst), ctypes.byref(n), _ptr(srcbuf), src.size)
    if r != 0:
        return r, b""
    return n.value, dst[:n.value].tobytes()


def ref_zstd_compress(data, level: int = 1) -> bytes:
    lib = _Lib.ref()
    src = _as_u8(data)
    cap = lib.ZSTD_compressBound(src.size)
    dst = np.zeros(cap + 16, dtype=np.uint8)
    r = lib.ZSTD_compress(_ptr(dst), cap, _ptr(src), src.size, level)
    assert not lib.ZSTD_isError(r)
    return dst[:r].tobytes()


def ref_zstd_decompress(comp, out_cap: int) -> tuple[int, bytes]:
    """The reference's ZSTD_decompress: (decoded size, or -1 when ZSTD_isError, bytes)."""
    lib = _Lib.ref()
    src = _as_u8(comp)
    srcbuf = np.zeros(src.size + 16, dtype=np.uint8)
    srcbuf[:src.size] = src
    dst = np.zeros(max(out_cap, 1) + 16, dtype=np.uint8)
    r = lib.ZSTD_decompress(_ptr(dst), out_cap, _ptr(srcbuf), src.size)
    if lib.ZSTD_isError(r):
        return -1, b""
    return int(r), dst[:r].tobytes()


def ref_zstd_compress_blocks(data, chunk: int, level: int = 1) -> bytes:
    """A multi-block frame: ZSTD_compressBegin + ZSTD_compressContinue per `chunk`
    bytes + ZSTD_compressEnd (zstd_compress.c), i.e. no content size in the header,
    one block per chunk, entropy tables and repeat offsets carried across blocks."""
    lib = _Lib.ref()
    src = _as_u8(data)
    cap = lib.ZSTD_compressBound(src.size) + 64 * (src.size // max(chunk, 1) + 2)
    dst = np.zeros(cap, dtype=np.uint8)
    cctx = lib.ZSTD_createCCtx()
    try:
        assert not lib.ZSTD_isError(lib.ZSTD_compressBegin(cctx, level))
        pos = out = 0
        base = src.ctypes.data
        while True:
            n = min(chunk, src.size - pos)
            last = pos + n >= src.size
            f = lib.ZSTD_compressEnd if last else lib.ZSTD_compressContinue
            r = f(cctx, ctypes.cast(dst.ctypes.data + out, _u8p), cap - out, ctypes.cast(base + pos, _u8p), n)
            assert not lib.ZSTD_isError(r), r
            out += r
            pos += n
            if last:
                break
    finally:
        lib.ZSTD_freeCCtx(cctx)
    return dst[:out].tobytes()


def ref_xxh64(data, seed: int = 0) -> int:
    src = _as_u8(data)
    return int(_Lib.ref().ZSTD_XXH64(_ptr(src), src.size, seed))
