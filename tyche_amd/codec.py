"""Device-resident batch codec on torch tensors (thin layer over the C ABI).

torch is only the plumbing here: it owns the HBM buffers and the stream; every
byte of codec work is done by the gfx950 kernels in libtyche_codec.so, reached
through ``tyche_compress_batch`` / ``tyche_decompress_batch``.

Layout in HBM: pages are rows of a (n, page_len) uint8
tensor; compressed pages are rows of a (n, slot) uint8 tensor whose slot is
``compress_bound(page_len)`` rounded up to 128 bytes, plus an int32 length per
row.  Only ``comp_len`` bytes of a slot are read or written by the kernels.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import LZ4_COMPRESSOR_ID

SLOT_ALIGN = 128


def compress_bound(n: int, compressor_id: int = LZ4_COMPRESSOR_ID) -> int:
    return int(_lib.load().tyche_compress_bound(compressor_id, n))


def slot_size(page_len: int, compressor_id: int = LZ4_COMPRESSOR_ID) -> int:
    b = compress_bound(page_len, compressor_id)
    return (b + SLOT_ALIGN - 1) // SLOT_ALIGN * SLOT_ALIGN


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def _check_pages(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (the codec runs only on the GPU)")
    if t.dtype != torch.uint8 or t.dim() != 2 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous 2-D uint8 tensor")


def compress_pages(pages: torch.Tensor, compressor_id: int = LZ4_COMPRESSOR_ID, level: int = 1,
                   out: torch.Tensor | None = None, out_len: torch.Tensor | None = None):
    """Compress every row of ``pages``; returns (slots, comp_len).

    comp_len[i] is LZ4_compress_default's return for row i (compressed bytes,
    0 on failure).  Asynchronous on the current stream.
    """
    _check_pages(pages, "pages")
    n, page_len = pages.shape
    slot = slot_size(page_len, compressor_id)
    if out is None:
        out = torch.empty((n, slot), dtype=torch.uint8, device=pages.device)
    if out_len is None:
        out_len = torch.empty((n,), dtype=torch.int32, device=pages.device)
    _check_pages(out, "out")
    b = _lib.Batch(count=n, src=_ptr(pages), src_stride=page_len, src_length=page_len, max_src_length=page_len,
                   dst=_ptr(out), dst_stride=out.shape[1], dst_capacity=out.shape[1], results=_ptr(out_len))
    rc = _lib.load().tyche_compress_batch(compressor_id, level, ctypes.byref(b), _stream_handle(pages.device))
    _lib.check(rc, "tyche_compress_batch")
    return out, out_len


def decompress_pages(slots: torch.Tensor, comp_len: torch.Tensor, page_len: int,
                     compressor_id: int = LZ4_COMPRESSOR_ID, out: torch.Tensor | None = None,
                     rv: torch.Tensor | None = None, max_comp_len: int = 0):
    """Decompress row i of ``slots`` (comp_len[i] bytes) into a page_len row.

    rv[i] is LZ4_decompress_safe's return (decoded size, or -(consumed)-1).
    ``max_comp_len`` (optional) bounds comp_len for LDS sizing; 0 = slot width.
    """
    _check_pages(slots, "slots")
    if comp_len.dtype != torch.int32 or not comp_len.is_cuda:
        raise ValueError("comp_len must be a device int32 tensor")
    n = slots.shape[0]
    if out is None:
        out = torch.empty((n, page_len), dtype=torch.uint8, device=slots.device)
    if rv is None:
        rv = torch.empty((n,), dtype=torch.int32, device=slots.device)
    _check_pages(out, "out")
    cap = max_comp_len if max_comp_len > 0 else slots.shape[1]
    b = _lib.Batch(count=n, src=_ptr(slots), src_lengths=_ptr(comp_len), src_stride=slots.shape[1],
                   max_src_length=min(cap, slots.shape[1]), dst=_ptr(out), dst_stride=out.shape[1],
                   dst_capacity=page_len, results=_ptr(rv))
    rc = _lib.load().tyche_decompress_batch(compressor_id, ctypes.byref(b), _stream_handle(slots.device))
    _lib.check(rc, "tyche_decompress_batch")
    return out, rv


def decompress_ragged(stream: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor, capacities: torch.Tensor,
                      out: torch.Tensor, out_offsets: torch.Tensor, rv: torch.Tensor, max_src_length: int,
                      max_capacity: int, compressor_id: int = LZ4_COMPRESSOR_ID):
    """General form: page i = stream[offsets[i] : offsets[i]+lengths[i]] -> out[out_offsets[i] : +capacities[i]]."""
    b = _lib.Batch(count=offsets.numel(), src=_ptr(stream), src_offsets=_ptr(offsets), src_lengths=_ptr(lengths),
                   max_src_length=max_src_length, dst=_ptr(out), dst_offsets=_ptr(out_offsets),
                   dst_capacities=_ptr(capacities), dst_capacity=max_capacity, results=_ptr(rv))
    rc = _lib.load().tyche_decompress_batch(compressor_id, ctypes.byref(b), _stream_handle(stream.device))
    _lib.check(rc, "tyche_decompress_batch")
    return out, rv


def compress_ragged(src: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor, out: torch.Tensor,
                    out_offsets: torch.Tensor, capacities: torch.Tensor, results: torch.Tensor, max_src_length: int,
                    compressor_id: int = LZ4_COMPRESSOR_ID, level: int = 1):
    b = _lib.Batch(count=offsets.numel(), src=_ptr(src), src_offsets=_ptr(offsets), src_lengths=_ptr(lengths),
                   max_src_length=max_src_length, dst=_ptr(out), dst_offsets=_ptr(out_offsets),
                   dst_capacities=_ptr(capacities), results=_ptr(results))
    rc = _lib.load().tyche_compress_batch(compressor_id, level, ctypes.byref(b), _stream_handle(src.device))
    _lib.check(rc, "tyche_compress_batch")
    return out, results


def pagegen(n: int, page_len: int, seed: int = 20170303, first: int = 0, dist: int = 0,
            device: torch.device | str = "cuda", out: torch.Tensor | None = None) -> torch.Tensor:
    """Synthetic database pages straight into HBM (tyche_amd/csrc/pagegen.h)."""
    dev = torch.device(device)
    if out is None:
        out = torch.empty((n, page_len), dtype=torch.uint8, device=dev)
    rc = _lib.load().tyche_pagegen(_ptr(out), out.shape[1], page_len, seed, first, n, dist, _stream_handle(dev))
    _lib.check(rc, "tyche_pagegen")
    return out
