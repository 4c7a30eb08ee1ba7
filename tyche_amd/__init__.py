"""tyche_amd -- MI355X-native batched page codec for tyche's compressed-offload path.

The product is libtyche_codec.so (gfx950 HIP kernels + the C ABI in
include/tyche_codec.h).  This package is the Python face of that ABI:

* ``tyche_amd.codec``  -- device-resident batch compress/decompress on torch tensors
* ``tyche_amd.buffer`` -- the Buffer entry points (buffer__compress / buffer__decompress)
* ``tyche_amd.sharding`` -- per-rank page partitioning for multi-GPU runs
"""
from ._lib import (COMPRESSOR_IDS, E_BAD_ARGS, E_BUFFER_ALREADY_COMPRESSED, E_BUFFER_ALREADY_DECOMPRESSED,
                   E_BUFFER_COMPRESSION_PROBLEM, E_BUFFER_MISSING_DATA, E_BUFFER_NOT_FOUND, E_DEVICE, E_OK,
                   LZ4_COMPRESSOR_ID, NO_COMPRESSOR_ID, ZLIB_COMPRESSOR_ID, ZSTD_COMPRESSOR_ID, load)

__all__ = ["COMPRESSOR_IDS", "E_BAD_ARGS", "E_BUFFER_ALREADY_COMPRESSED", "E_BUFFER_ALREADY_DECOMPRESSED",
           "E_BUFFER_COMPRESSION_PROBLEM", "E_BUFFER_MISSING_DATA", "E_BUFFER_NOT_FOUND", "E_DEVICE", "E_OK",
           "LZ4_COMPRESSOR_ID", "NO_COMPRESSOR_ID", "ZLIB_COMPRESSOR_ID", "ZSTD_COMPRESSOR_ID", "load"]
