"""Build recipe for libtyche_codec.so (gfx950 code objects + the C ABI).

hipcc compiles each .hip file to an object (in parallel) and links one shared
library in-tree, next to this file, so it travels to the GPU box with the repo
snapshot.  No JIT cache, no site-packages install.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "..", "build", "tyche_amd")
LIB = os.path.join(HERE, "libtyche_codec.so")
SOURCES = ["engine.hip", "lz4_decode.hip", "lz4_decode_lane.hip", "lz4_decode_lc.hip", "lz4_encode.hip", "zlib_inflate.hip", "zstd_decode.hip", "zstd_encode.hip", "zlib_deflate.hip", "pagegen.hip",
           "errno_guard.hip"]   # errno_guard last: its constructor runs after the code-object registrations
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-variable",
         "-munsafe-fp-atomics", "-I" + os.path.join(HERE, "..", "include")]
# The encoders and the zstd decoder read LDS as aligned dwords (lz_parse.h, ld64): LLVM's IR
# load/store vectorizer would fuse neighbouring dwords into ds_read_b64/b128 at
# 4-byte-aligned addresses, which the LDS replays at ~64 cycles per instruction.
# Without it, pairs still become ds_read2_b32 (4-byte alignment suffices).
# superseded large-batch LZ4 decoders (round-2/3 lane kernels, the round-4 quad kernel): only in the
# A/B build, libtyche_codec_legacy_decoders.so (build(legacy=True)), never in the product library
LEGACY_SOURCES = ["legacy/lz4_decode_lane_legacy.hip", "legacy/lz4_decode_quad.hip"]
NO_LSV = ["-mllvm", "-amdgpu-load-store-vectorizer=false"]
SOURCE_FLAGS = {"lz4_encode.hip": NO_LSV, "zstd_encode.hip": NO_LSV, "zlib_deflate.hip": NO_LSV, "zstd_decode.hip": NO_LSV}


def kernel_sources_digest() -> str:
    """sha256 (first 16 hex digits) over the kernel sources (csrc/*.hip, csrc/*.h and the ABI
    header): PMC traffic summaries record it (tools/pmc_traffic.py) so that bench.py can tell a
    summary of the code it runs from a stale one."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    for f in files:
        h.update(f.encode())
        h.update(open(os.path.join(CSRC, f), "rb").read())
    h.update(open(os.path.join(HERE, "..", "include", "tyche_codec.h"), "rb").read())
    return h.hexdigest()[:16]


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build(force: bool = False, verbose: bool = False, profile: bool = False, ablate: int = 0,
          eablate: int = 0, defines: tuple = (), legacy: bool = False) -> str:
    """profile=True builds the diagnostic variant (per-phase cycle stamps, -DTYCHE_PROFILE)
    as libtyche_codec_prof.so; it is never loaded by the product path."""
    if legacy:
        defines = tuple(defines) + ("TYCHE_LEGACY_DECODERS",)
    tag = ("_prof" if profile else "") + (f"_abl{ablate}" if ablate else "") + (f"_eabl{eablate}" if eablate else "") + \
        "".join("_" + d.replace("TYCHE_", "").replace("=", "").lower() for d in defines)   # A/B variant libraries
    build_dir = BUILD + tag
    lib_path = LIB.replace(".so", tag + ".so")
    flags = FLAGS + (["-DTYCHE_PROFILE"] if profile else []) + ([f"-DTYCHE_ABLATE={ablate}"] if ablate else []) + \
        ([f"-DTYCHE_EABLATE={eablate}"] if eablate else []) + ["-D" + d for d in defines]
    os.makedirs(build_dir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]   # (legacy/ has none)
    headers.append(os.path.join(HERE, "..", "include", "tyche_codec.h"))
    objs = []
    jobs = []
    sources = SOURCES[:-1] + (LEGACY_SOURCES if legacy else []) + SOURCES[-1:]   # errno_guard stays last
    for src in sources:
        s = os.path.join(CSRC, src)
        o = os.path.join(build_dir, src.replace("/", "_").replace(".hip", ".o"))
        objs.append(o)
        if force or not _newer(o, [s] + headers):
            jobs.append([HIPCC] + flags + SOURCE_FLAGS.get(src, []) + ["-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)

    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            list(ex.map(run, jobs))
    if force or jobs or not _newer(lib_path, objs):
        run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib_path] + objs)
    return lib_path


def build_tools(verbose: bool = False) -> list:
    """tools/bin/{cycle,stress}: C harnesses over the C ABI (tools/cycle.c: the tyche-shaped
    sweep/restore cycle; tools/stress.c: hundreds of concurrent Buffer API callers)."""
    root = os.path.abspath(os.path.join(HERE, ".."))
    out_dir = os.path.join(root, "tools", "bin")
    os.makedirs(out_dir, exist_ok=True)
    outs = []
    for name in ("cycle", "cycle_live", "stress", "latency"):
        src = os.path.join(root, "tools", name + ".c")
        out = os.path.join(out_dir, name)
        outs.append(out)
        deps = [src, os.path.join(root, "include", "tyche_codec.h"), os.path.join(CSRC, "pagegen.h"), LIB]
        if _newer(out, deps):
            continue
        cmd = ["gcc", "-O2", "-g", "-rdynamic", "-std=gnu99", "-Wall", "-o", out, src, "-I" + os.path.join(root, "include"),
               "-L" + HERE, "-ltyche_codec", "-Wl,-rpath,$ORIGIN/../../tyche_amd", "-lpthread"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    return outs


if __name__ == "__main__":
    import sys
    abl = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--ablate=")]
    eabl = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--eablate=")]
    print(build(force="--force" in sys.argv, verbose=True, profile="--profile" in sys.argv,
                ablate=abl[0] if abl else 0, eablate=eabl[0] if eabl else 0, legacy="--legacy" in sys.argv))
