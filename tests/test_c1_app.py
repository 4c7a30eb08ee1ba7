"""C1 (BASELINE.json configs[0]): the reference tyche application, unmodified,
linked against libtyche_codec.so instead of its own src/buffer.c.

integration/Makefile compiles /root/reference/src/{list,options,manager,error,
io,tests,tyche}.c + lz4/lz4.c into integration/_app/tyche (and tyche_q, the
same with a delayed free() for the reference's clock_hand use-after-free,
SURVEY §4) at build time, where the reference tree exists; the binaries travel
to the GPU box like the .so.  The page directory is rebuilt from the committed
fixture (tests/golden/lz4_sample.npz: the reference's LZ4 encodings of the 60
sample_data pages plus their SHA-256), so nothing reads /root/reference at run
time.

* CPU: loading the library leaves errno == 0 (the reference's io.c:89-93 tests
  errno after opendir), and the app starts, scans its pages and reaches the
  codec, which refuses loudly without a GPU.
* GPU: `tyche -t compression -c lz4|zlib|zstd` (src/tests.c:340-443) passes
  through the GPU codec, and a short `-c lz4 -p sample_data/16k -w 1` run
  compresses and restores pages through list.c's own callers
  (list.c:1051, 572).
"""
import hashlib
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden

APP = os.path.join(ROOT, "integration", "_app", "tyche")
APP_Q = os.path.join(ROOT, "integration", "_app", "tyche_q")
LIB_DIR = os.path.join(ROOT, "tyche_amd")


def _need(path):
    if not os.path.exists(path):
        pytest.skip(f"{os.path.relpath(path, ROOT)} not built (build() makes it where /root/reference exists)")


@pytest.fixture(scope="module")
def sample_dir(tmp_path_factory, oracle_mod):
    """sample_data/ rebuilt from the fixture: every page decoded by the oracle and checked by digest."""
    g = load_golden("lz4_sample.npz")
    root = tmp_path_factory.mktemp("sample_data")
    for i, name in enumerate(g["names"]):
        comp = g["comp"][g["comp_off"][i]:g["comp_off"][i] + g["comp_len"][i]]
        r, page = oracle_mod.lz4_decompress(comp, int(g["size"][i]))
        assert r == g["size"][i] and hashlib.sha256(page).digest() == g["digest"][i].tobytes(), name
        path = root / str(name)
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_bytes(page)
    return root


def _run(args, timeout):
    p = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
    return p.returncode, p.stdout.decode(errors="replace")


def test_library_load_leaves_errno_zero(tmp_path):
    """A program linked against the engine reaches main() with errno == 0 (C's start-up state)."""
    src = tmp_path / "probe.c"
    src.write_text('#include <errno.h>\n#include <stdio.h>\nint main(void){printf("errno=%d\\n", errno);return 0;}\n')
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-o", str(exe), str(src), "-Wl,--no-as-needed", "-L" + LIB_DIR, "-ltyche_codec",
                           "-Wl,-rpath," + LIB_DIR])
    out = subprocess.check_output([str(exe)]).decode()
    assert out.strip() == "errno=0", out


def test_reference_app_starts_without_gpu(sample_dir):
    """The unmodified app gets past option parsing and the page scan (io.c) and into the codec
    test; without a GPU the engine refuses with TYCHE_E_DEVICE (199) instead of running on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (the GPU tests below cover the full run)")
    _need(APP)
    rc, out = _run([APP, "-t", "compression", "-c", "lz4", "-p", str(sample_dir / "16k")], 60)
    assert "File/directory not found" not in out, out
    assert "Test 3: passed" in out, out
    assert "buffer__compress: 199" in out, out


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["lz4", "zlib", "zstd"])
def test_reference_app_compression_test(sample_dir, codec):
    """tests__compression (src/tests.c:340-443): Test 4 round-trips the Lorem page through
    buffer__compress / buffer__decompress, i.e. through the GPU engine."""
    _need(APP)
    rc, out = _run([APP, "-t", "compression", "-c", codec, "-p", str(sample_dir / "16k")], 90)
    # the app always quits non-zero after a test (manager.c:105-109: exit(E_GENERIC))
    assert "Test 'compression': all passed!" in out, out
    assert rc == 1, (rc, out)
    m = re.search(r"Compression gave an OK response\..*comp_length is (\d+) bytes", out)
    assert m and 0 < int(m.group(1)) < 4096, out


@pytest.mark.gpu
def test_reference_app_benchmark_run_lz4(sample_dir):
    """A short benchmark run of the reference app (`-c lz4 -p sample_data/16k -w 1 -d 3`, a 20 % fixed raw
    ratio of 512,000 bytes so the sweeper has to compress): its compressor pool (one thread per CPU, 256
    on the GPU box) and its restore path call the engine, and pages are compressed and restored.

    Two defects of the reference's own list code can keep the process from exiting, so the harness
    watchdog (integration/quarantine.c, TYCHE_APP_WATCHDOG) dumps every thread's stack and exits 3 after
    15 s; the run then counts only if the dump shows one of them and no thread inside the engine:
      * shutdown: list__destroy "stops" the compressors by setting runnable = 1 (list.c:972-973) and
        joins them forever (list.c:979-980) -- the results block has been printed by then;
      * mid-run: list__sweep's clock scan (list.c:795-816) spins until it meets an unpopular raw buffer
        that is not already pending, and on a 20-page data set there may be none, so the worker waits in
        list__search (list.c:509-522); the app's status line (manager.c:193) still shows its counters."""
    _need(APP_Q)
    env = dict(os.environ, TYCHE_APP_WATCHDOG="15")
    # the reference's list code is racy: a run can wedge before its first restore; up to
    # three runs, the first that restored anything is checked
    for attempt in range(3):
        p = subprocess.run([APP_Q, "-c", "lz4", "-p", str(sample_dir / "16k"), "-w", "1", "-d", "3", "-m", "512000",
                            "-f", "20"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=90, env=env)
        out, err = p.stdout.decode(errors="replace"), p.stderr.decode(errors="replace")
        if re.search(r"Restorations\s*:\s*[1-9]", out) or re.search(r"\(([1-9][\d.,]*)\S? Res\)", err):
            break
    comp = re.search(r"Compressions\s*:\s*([\d,]+) compressions", out)
    rest = re.search(r"Restorations\s*:\s*([\d,]+) restorations", out)
    if comp and rest:
        comps, rests = int(comp.group(1).replace(",", "")), int(rest.group(1).replace(",", ""))
    else:
        status = re.findall(r"([\d.,]+)(\S?) Comps \(([\d.,]+)(\S?) Res\)", err)
        assert status, (p.returncode, out[-2000:], err[-2000:])
        scale = {"": 1, "K": 1e3, "M": 1e6, "B": 1e9}
        comps = float(status[-1][0].replace(",", "")) * scale.get(status[-1][1], 1)
        rests = float(status[-1][2].replace(",", "")) * scale.get(status[-1][3], 1)
    assert comps > 0 and rests > 0, (comps, rests, out[-2000:])
    if p.returncode == 3:
        dump = err[err.find("--- thread"):]
        assert "--- thread" in dump, err[-2000:]
        assert "buffer__compress" not in dump and "buffer__decompress" not in dump   # no thread in the engine
        if comp and rest:
            assert "list__destroy" in dump, dump[-3000:]    # the reference's shutdown hang
        else:
            assert "list__sweep" in dump, dump[-3000:]      # the reference's sweep wedge
    else:
        assert p.returncode == 0 and comp and rest, (p.returncode, out[-2000:], err[-2000:])
