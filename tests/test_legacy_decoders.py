"""The superseded large-batch LZ4 decoders (round-2/3 lane kernels, the round-4 quad kernel), kept
for A/B timing only in libtyche_codec_legacy_decoders.so (tyche_amd/_build.py: build(legacy=True)),
never in the product library.  Deselected unless TYCHE_CODEC_LIB names that build:

    python -c "from tyche_amd import _build; _build.build(legacy=True)"
    TYCHE_CODEC_LIB=tyche_amd/libtyche_codec_legacy_decoders.so python -m pytest tests/test_legacy_decoders.py -m gpu
"""
import numpy as np
import pytest

from test_gpu_lz4 import ragged_decode, tc  # noqa: F401
from test_gpu_lz4 import test_decode_jump_path_page_kinds as page_kinds
from test_gpu_lz4 import test_decode_lane_path_fixtures as lane_fixtures

pytestmark = [pytest.mark.gpu, pytest.mark.legacy]


@pytest.mark.parametrize("lb,ring", [(1, 128), (1, 160), (1, 192), (1, 256), (0, 256), (0, 128)])
def test_decode_lane_kernels_all_rings(tc, oracle_mod, knobs, lb, ring):
    """Every lane-per-page kernel variant (LZ4_LANE_LB=1: the stream through a per-lane line buffer,
    the default, at each ring size; 0: the round-2 ring kernel), selected in-process with
    tyche_set_knob and forced on every batch size (LZ4_LANE_MIN=0): the fixtures with their exact
    return values, and seeded corruptions against the restated LZ4_decompress_safe."""
    knobs(LZ4_LC=0, LZ4_LANE_LB=lb, LZ4_LANE_RING=ring, LZ4_LANE_MIN=0)
    lane_fixtures(tc, 1)
    rng = np.random.default_rng(1000 + ring + lb)
    pages = oracle_mod.pagegen(256, 16384, seed=9, first=ring, dist=0)
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
        if r > 0 and i % 4 in (0, 3):   # untouched streams (a flipped one may hold an offset-0 match: undefined bytes)
            assert outs[i][:r] == want[:r], i


@pytest.mark.parametrize("ring,far", [(1024, 8), (1024, 6), (512, 8), (512, 6), (2048, 8)])
def test_decode_quad_kernel_variants(tc, oracle_mod, knobs, ring, far):
    """The quad-per-page chunked decoder (lz4_decode_quad.hip) at every ring / far-entry size,
    forced on every batch size (LZ4_QUAD=1, LZ4_LANE_MIN=0): the fixtures with their exact return
    values, seeded corruptions against the restated LZ4_decompress_safe, and pages built for its
    slow path (incompressible, long literal runs, long and self-overlapping matches)."""
    knobs(LZ4_QUAD=1, LZ4_QUAD_RING=ring, LZ4_QUAD_FAR=far, LZ4_LANE_MIN=0)
    lane_fixtures(tc, 1)
    rng = np.random.default_rng(2000 + ring + far)
    pages = oracle_mod.pagegen(256, 16384, seed=11, first=ring + far, dist=0)
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
        page_kinds(tc, oracle_mod, plen, 300)
