"""ctypes binding of libtyche_codec.so -- the C ABI declared in include/tyche_codec.h.

The library is the product: HIP kernels for gfx950 plus the drop-in
buffer__compress / buffer__decompress entry points.  Loading fails loudly if the
in-tree .so is missing; there is no Python or CPU fallback for any codec call.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TYCHE_CODEC_LIB") or os.path.join(HERE, "libtyche_codec.so")
HEADER = os.path.join(HERE, "..", "include", "tyche_codec.h")

# compressor IDs, src/globals.h:16-19
NO_COMPRESSOR_ID = 0
LZ4_COMPRESSOR_ID = 1
ZLIB_COMPRESSOR_ID = 2
ZSTD_COMPRESSOR_ID = 3
COMPRESSOR_IDS = {"none": 0, "lz4": 1, "zlib": 2, "zstd": 3}

# error codes, src/globals.h:35-58 (+ the engine's own device error)
E_OK = 0
E_GENERIC = 1
E_BUFFER_NOT_FOUND = 120
E_BUFFER_MISSING_DATA = 123
E_BUFFER_ALREADY_COMPRESSED = 124
E_BUFFER_ALREADY_DECOMPRESSED = 125
E_BUFFER_COMPRESSION_PROBLEM = 126
E_NO_MEMORY = 150
E_BAD_ARGS = 190
E_DEVICE = 199
ALL_DEVICES = -1        # tyche_set_device: spread host work over the device set (TYCHE_ALL_DEVICES)

RESULT_TOO_LARGE = -(2 ** 31)

# buffer flags, src/buffer.h:23-33
FLAG_COMPRESSING = 1 << 5
FLAG_COMPRESSED = 1 << 6


class PthreadMutex(ctypes.Structure):
    # glibc x86_64 pthread_mutex_t: 40 bytes, 8-byte aligned
    _fields_ = [("_opaque", ctypes.c_int64 * 5)]


class Buffer(ctypes.Structure):
    """struct buffer, src/buffer.h:39-58 (same field order, types and padding)."""


Buffer._fields_ = [
    ("next", ctypes.POINTER(Buffer)),
    ("id", ctypes.c_uint32),
    ("ref_count", ctypes.c_uint16),
    ("flags", ctypes.c_int),
    ("popularity", ctypes.c_uint8),
    ("lock", PthreadMutex),
    ("comp_cost", ctypes.c_uint32),
    ("comp_hits", ctypes.c_uint16),
    ("data_length", ctypes.c_uint32),
    ("comp_length", ctypes.c_uint32),
    ("data", ctypes.c_void_p),
]


class Batch(ctypes.Structure):
    """tyche_batch_t (include/tyche_codec.h)."""

    _fields_ = [
        ("count", ctypes.c_size_t),
        ("src", ctypes.c_void_p),
        ("src_offsets", ctypes.c_void_p),
        ("src_lengths", ctypes.c_void_p),
        ("src_stride", ctypes.c_uint64),
        ("src_length", ctypes.c_uint32),
        ("max_src_length", ctypes.c_uint32),
        ("dst", ctypes.c_void_p),
        ("dst_offsets", ctypes.c_void_p),
        ("dst_capacities", ctypes.c_void_p),
        ("dst_stride", ctypes.c_uint64),
        ("dst_capacity", ctypes.c_uint32),
        ("results", ctypes.c_void_p),
    ]


_BufP = ctypes.POINTER(Buffer)
_vpp = ctypes.POINTER(ctypes.c_void_p)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i32p = ctypes.POINTER(ctypes.c_int32)
_intp = ctypes.POINTER(ctypes.c_int)

# every function declared in include/tyche_codec.h: name -> (restype, argtypes)
SIGNATURES = {
    "buffer__initialize": (ctypes.c_int, [ctypes.POINTER(_BufP), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                          ctypes.c_char_p]),
    "buffer__destroy": (None, [_BufP, ctypes.c_bool]),
    "buffer__lock": (None, [_BufP]),
    "buffer__unlock": (None, [_BufP]),
    "buffer__release_pin": (None, [_BufP]),
    "buffer__compress": (ctypes.c_int, [_BufP, _vpp, ctypes.c_int, ctypes.c_int]),
    "buffer__decompress": (ctypes.c_int, [_BufP, ctypes.c_int]),
    "buffer__copy": (None, [_BufP, _BufP, ctypes.c_bool]),
    "tyche_buffers_compress": (ctypes.c_int, [ctypes.POINTER(_BufP), _vpp, _intp, ctypes.c_size_t, ctypes.c_int,
                                              ctypes.c_int]),
    "tyche_buffers_decompress": (ctypes.c_int, [ctypes.POINTER(_BufP), _intp, ctypes.c_size_t, ctypes.c_int]),
    "tyche_compress_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(Batch), ctypes.c_void_p]),
    "tyche_decompress_batch": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(Batch), ctypes.c_void_p]),
    "tyche_compress_bound": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_uint32]),
    "tyche_compress_host": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, _vpp, _u32p, _vpp, _u32p,
                                           _i32p]),
    "tyche_decompress_host": (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, _vpp, _u32p, _vpp, _u32p, _i32p]),
    "tyche_restore_queue_start": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "tyche_restore_queue_stop": (None, []),
    "tyche_buffer_restore": (ctypes.c_int, [_BufP, ctypes.c_int]),
    "tyche_restore_queue_stats": (None, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "tyche_restore_queue_hist": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "tyche_device_count": (ctypes.c_int, []),
    "tyche_set_device": (ctypes.c_int, [ctypes.c_int]),
    "tyche_active_devices": (ctypes.c_int, []),
    "tyche_plan_split": (ctypes.c_size_t, [ctypes.c_size_t, _u32p, ctypes.c_int, ctypes.c_uint64,
                                           ctypes.POINTER(ctypes.c_size_t)]),
    "tyche_host_profile": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "tyche_set_knob": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_long]),
    "tyche_clear_knob": (ctypes.c_int, [ctypes.c_char_p]),
    "tyche_last_error": (ctypes.c_char_p, []),
    "tyche_device_ready": (ctypes.c_int, []),
    "tyche_pagegen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                     ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p]),
}

_lib = None


def load(build_if_missing: bool = False) -> ctypes.CDLL:
    """Loads the in-tree libtyche_codec.so; raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build_if_missing:
            raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`"
                               " (the codec has no CPU fallback)")
        from . import _build
        _build.build()
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def set_knob(name: str, value: int) -> None:
    """In-process override of a TYCHE_<name> switch (include/tyche_codec.h: tyche_set_knob)."""
    check(load().tyche_set_knob(name.encode(), int(value)), f"tyche_set_knob({name})")


def clear_knob(name: str) -> None:
    check(load().tyche_clear_knob(name.encode()), f"tyche_clear_knob({name})")


def last_error() -> str:
    return (load().tyche_last_error() or b"").decode(errors="replace")


class DeviceError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != E_OK:
        raise DeviceError(f"{what} failed with code {rc}: {last_error()}")
