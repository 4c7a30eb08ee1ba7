import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP kernels through the C ABI")
    config.addinivalue_line("markers", "legacy: superseded decoders, only in the A/B library build (test_legacy_decoders.py)")


def pytest_collection_modifyitems(config, items):
    """Legacy-decoder tests run only against the library that contains those kernels."""
    if "legacy" in os.environ.get("TYCHE_CODEC_LIB", ""):
        return
    keep = [it for it in items if it.get_closest_marker("legacy") is None]
    if len(keep) != len(items):
        config.hook.pytest_deselected(items=[it for it in items if it.get_closest_marker("legacy") is not None])
        items[:] = keep


def load_golden(name: str):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def unpack(data: np.ndarray, offs: np.ndarray, lens: np.ndarray, i: int) -> bytes:
    return data[offs[i]:offs[i] + lens[i]].tobytes()


@pytest.fixture
def knobs():
    """Sets engine switches for one test through tyche_set_knob (read on every launch) and
    drops the overrides afterwards: knobs(ZLIB_PAR=0, LZ4_LANE_MIN=0)."""
    from tyche_amd import _lib
    names = set()

    def setter(**kv):
        for k, v in kv.items():
            _lib.set_knob(k, int(v))
            names.add(k)
    yield setter
    for k in names:
        _lib.clear_knob(k)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build(ref=False) if not os.path.exists(O.ORACLE_SO) else None
    return O
