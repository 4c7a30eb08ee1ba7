"""CPU check of the chunked lane-per-page LZ4 decoder's algorithm (tyche_amd/csrc/lz4_lc_core.h,
the per-lane code of lz4_decode_lc.hip) through its host emulator tools/lc_emul.cpp, against the
restated LZ4_decompress_safe (oracle, lz4.c:1251): the reference-generated, sample and malformed
fixtures, seeded corruptions, and the page kinds that exercise split records (incompressible pages,
zero and short-period pages, 64 KiB-1 pages) -- exact return values, and the bytes wherever the
reference's output is defined.  The GPU parity tests (test_gpu_lz4.py::test_decode_lc_kernel_variants)
run the kernel itself on the same kinds of input."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden, unpack

LIB = os.path.join(ROOT, "tools", "bin", "liblcemul.so")
SRC = os.path.join(ROOT, "tools", "lc_emul.cpp")
CORE = [os.path.join(ROOT, "tyche_amd", "csrc", f) for f in ("lz4_lc_core.h", "byte_funnel.h")]


@pytest.fixture(scope="module", params=[0, 1], ids=["far32", "far16"])
def emul(request):
    """The emulator built as each kernel build is: far match parts of up to 32 bytes (two far
    registers per record slot) or, LC_FAR16=1 (the default), of up to 16 bytes (one register;
    longer far matches continue in the next record)."""
    far16 = request.param
    lib_path = LIB.replace(".so", "_f%d.so" % far16)
    if not os.path.exists(lib_path) or any(os.path.getmtime(f) > os.path.getmtime(lib_path) for f in [SRC] + CORE):
        os.makedirs(os.path.dirname(lib_path), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-DLC_FAR16=%d" % far16, "-o", lib_path, SRC])
    lib = ctypes.CDLL(lib_path)

    def dec(s, cap, ring):
        buf = (ctypes.c_uint8 * max(len(s), 1)).from_buffer_copy(s if s else b"\0")
        out = (ctypes.c_uint8 * (cap + 64))()
        r = lib.lc_emul_decode(buf, len(s), out, cap, ring)
        return r, bytes(out[:max(r, 0)])
    return dec


def _cases(O):
    gm, gg, gs = load_golden("lz4_malformed.npz"), load_golden("lz4_generated.npz"), load_golden("lz4_sample.npz")
    cases = [(unpack(gm["comp"], gm["comp_off"], gm["comp_len"], i), int(gm["cap"][i]), bool(gm["defined"][i]))
             for i in range(len(gm["cap"]))]
    cases += [(unpack(gg["comp"], gg["comp_off"], gg["comp_len"], i), int(gg["meta"][i][1]), True)
              for i in range(len(gg["digest"]))]
    cases += [(unpack(gs["comp"], gs["comp_off"], gs["comp_len"], i), int(gs["size"][i]), True)
              for i in range(len(gs["digest"]))]
    rng = np.random.default_rng(77)
    pages = O.pagegen(200, 16384, seed=9, dist=0)
    for i in range(200):
        c = bytearray(O.lz4_compress(pages[i].tobytes()))
        if i % 4 == 1:
            c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
        elif i % 4 == 2:
            c = c[: int(rng.integers(1, len(c)))]
        cases.append((bytes(c), 16384 if i % 4 != 3 else int(rng.integers(100, 16384)), i % 4 in (0, 3)))
    g = np.random.default_rng(5)
    for plen in (8192, 16384, 32768, 65535):
        for kind in range(5):
            if kind == 0:
                p = g.integers(0, 256, plen, dtype=np.uint8)
            elif kind == 1:
                p = np.zeros(plen, np.uint8)
            elif kind == 2:
                per = int(g.integers(1, 40))
                p = np.tile(g.integers(0, 256, per, dtype=np.uint8), plen // per + 1)[:plen]
            elif kind == 3:
                p = O.pagegen(1, (plen + 4095) // 4096 * 4096, seed=plen, dist=int(g.integers(0, 6)))[0][:plen]
            else:
                p = np.tile(g.integers(0, 256, 24, dtype=np.uint8), plen // 24 + 1)[:plen].copy()
                noise = g.integers(0, plen, plen // 97)
                p[noise] = g.integers(0, 256, noise.size, dtype=np.uint8)
            cases.append((O.lz4_compress(p.tobytes()), plen, True))
    return cases


@pytest.mark.parametrize("ring", [128, 160, 192, 256])
def test_lc_algorithm_vs_oracle(emul, oracle_mod, ring):
    for k, (s, cap, defined) in enumerate(_cases(oracle_mod)):
        r, out = emul(s, cap, ring)
        orv, want = oracle_mod.lz4_decompress(s, cap)
        assert r == orv, (k, r, orv, len(s), cap)
        if defined and r >= 0:
            assert out == want[:r], k
