"""The C ABI (include/tyche_codec.h) without a GPU: the library loads, exports
every declared symbol, keeps the reference's Buffer layout (src/buffer.h:39-58)
and error behaviour (src/buffer.c:159-281) for every path that does not reach
the codec, and refuses codec work loudly when no gfx950 device is present."""
import ctypes
import os
import re
import subprocess
import textwrap

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tyche_codec.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:[\w\s\*]+?)\b(\w+)\s*\([^;{]*\)\s*;", text, flags=re.M)
    return sorted(set(n for n in names if not n.startswith("__")))


def test_library_exports_every_declared_symbol():
    from tyche_amd import _lib
    lib = _lib.load()
    decl = declared_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), name
    # the Python binding covers the same set
    assert set(decl) == set(_lib.SIGNATURES), set(decl) ^ set(_lib.SIGNATURES)


def test_library_has_no_cpu_codec_inside():
    """The product library links no CPU LZ4/zlib/zstd: none of the vendored codec symbols are defined."""
    from tyche_amd import _lib
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    for sym in ("LZ4_compress_default", "LZ4_decompress_safe", "compress2", "uncompress", "ZSTD_compress",
                "oracle_lz4_compress"):
        assert not re.search(rf"\b{sym}\b", out), sym


def test_buffer_struct_layout_matches_c(tmp_path):
    """ctypes Buffer == the header's struct buffer (field offsets + size), checked with gcc."""
    from tyche_amd._lib import Buffer
    src = tmp_path / "probe.c"
    src.write_text(textwrap.dedent(f"""
        #include <stdio.h>
        #include <stddef.h>
        #include "{HEADER}"
        int main(void) {{
            printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(Buffer),
                offsetof(Buffer, next), offsetof(Buffer, id), offsetof(Buffer, ref_count), offsetof(Buffer, flags),
                offsetof(Buffer, popularity), offsetof(Buffer, lock), offsetof(Buffer, comp_cost),
                offsetof(Buffer, comp_hits), offsetof(Buffer, data_length), offsetof(Buffer, comp_length),
                offsetof(Buffer, data));
            return 0;
        }}"""))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(Buffer)] + [getattr(Buffer, f).offset for f in
                                      ("next", "id", "ref_count", "flags", "popularity", "lock", "comp_cost",
                                       "comp_hits", "data_length", "comp_length", "data")]
    assert got == want


def test_buffer_struct_matches_reference_header(tmp_path):
    """Same layout as the reference's own src/buffer.h (where the reference tree exists)."""
    ref = "/root/reference/src/buffer.h"
    if not os.path.exists(ref):
        pytest.skip("reference tree not present")
    src = tmp_path / "probe.c"
    src.write_text(textwrap.dedent(f"""
        #include <pthread.h>
        #include <stdio.h>
        #include <stddef.h>
        #include "{ref}"
        int main(void) {{
            printf("%zu %zu %zu %zu %zu\\n", sizeof(Buffer), offsetof(Buffer, comp_cost),
                   offsetof(Buffer, data_length), offsetof(Buffer, comp_length), offsetof(Buffer, data));
            return 0;
        }}"""))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    from tyche_amd._lib import Buffer
    assert got == [ctypes.sizeof(Buffer), Buffer.comp_cost.offset, Buffer.data_length.offset,
                   Buffer.comp_length.offset, Buffer.data.offset]


def test_precheck_order_without_device():
    """buffer__compress / buffer__decompress argument checks (buffer.c:161-174, 229-240), no codec call."""
    from tyche_amd import buffer as B
    from tyche_amd._lib import (E_BUFFER_ALREADY_COMPRESSED, E_BUFFER_ALREADY_DECOMPRESSED,
                                E_BUFFER_MISSING_DATA, E_OK, LZ4_COMPRESSOR_ID, NO_COMPRESSOR_ID)
    buf = B.new_buffer(b"x" * 100, id=7)
    # NO compressor: comp_length = data_length, OK, data untouched
    rv, out = B.buffer__compress(buf, NO_COMPRESSOR_ID)
    assert rv == E_OK and out is None and buf.contents.comp_length == 100
    # already compressed
    rv, _ = B.buffer__compress(buf, LZ4_COMPRESSOR_ID)
    assert rv == E_BUFFER_ALREADY_COMPRESSED
    # NO decompress clears comp_length
    assert B.buffer__decompress(buf, NO_COMPRESSOR_ID) == E_OK and buf.contents.comp_length == 0
    assert B.buffer__decompress(buf, LZ4_COMPRESSOR_ID) == E_BUFFER_ALREADY_DECOMPRESSED
    # missing data
    empty = B.new_buffer(None, id=8)
    rv, _ = B.buffer__compress(empty, LZ4_COMPRESSOR_ID)
    assert rv == E_BUFFER_MISSING_DATA
    empty.contents.comp_length = 5
    assert B.buffer__decompress(empty, LZ4_COMPRESSOR_ID) == E_BUFFER_MISSING_DATA
    B.destroy(buf)
    B.destroy(empty, destroy_data=False)


def test_codec_refuses_without_gfx950():
    """No GPU here: the codec path reports an error instead of silently running on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from tyche_amd import buffer as B
    from tyche_amd import _lib
    buf = B.new_buffer(b"abcdefgh" * 512, id=1)
    rv, out = B.buffer__compress(buf, _lib.LZ4_COMPRESSOR_ID)
    assert rv != _lib.E_OK and out is None
    assert "device" in _lib.last_error().lower()
    assert buf.contents.comp_length == 0
    B.destroy(buf)


def test_buffer_initialize_from_file(tmp_path):
    """buffer__initialize's page_filespec path (buffer.c:88-106) and its argument rules."""
    from tyche_amd import _lib
    lib = _lib.load()
    page = tmp_path / "page"
    page.write_bytes(bytes(range(256)) * 32)
    bp = ctypes.POINTER(_lib.Buffer)()
    assert lib.buffer__initialize(ctypes.byref(bp), 3, 0, None, str(page).encode()) == _lib.E_OK
    assert bp.contents.data_length == 8192 and bp.contents.id == 3
    assert ctypes.string_at(bp.contents.data, 8192) == page.read_bytes()
    lib.buffer__destroy(bp, True)
    bp2 = ctypes.POINTER(_lib.Buffer)()
    assert lib.buffer__initialize(ctypes.byref(bp2), 3, 10, None, str(page).encode()) == _lib.E_BAD_ARGS
