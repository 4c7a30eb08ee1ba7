#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X.

Metric: GiB/s device-resident LZ4 compress+decompress of 1M x 16 KiB pages
(configs[1], "C2"), per GPU, weak scaling over 1/2/4/8 GPUs.  One step = one
compress pass + one decompress pass over the rank's 1,048,576 resident pages;
value = uncompressed bytes of all ranks' pages x steps / max-over-ranks wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C4]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--config C4 measures BASELINE configs[3] instead: LZ4 decompress-only of 8M x 8 KiB
pages, split over the ranks by contiguous page ranges (strong scaling).

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel, HIP events on
the codec's stream) and `cpu_baseline` (the reference's vendored LZ4 1.7.5 from
oracle/_ref, timed by oracle/_ref/cpu_baseline: C pthreads on every core the
process may use -- its affinity mask, capped by its cgroup CPU quota -- over a
bounded sample of the same pages).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tyche_amd import _lib, codec, runner  # noqa: E402

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
METRIC = "GiB/s device-resident LZ4 compress+decompress, 1M×16KiB pages, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pages", type=int, default=1 << 20, help="pages per GPU")
    ap.add_argument("--page-len", type=int, default=16384)
    ap.add_argument("--dist", type=int, default=0, help="pagegen distribution (0 = pg mix)")
    ap.add_argument("--seed", type=int, default=20170303)
    ap.add_argument("--cpu-pages", type=int, default=131072, help="CPU baseline sample (pages, at least 2048 per thread)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core the process may use (affinity, cgroup quota)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e-pages", type=int, default=32768, help="host-buffer (PCIe-inclusive) sample; 0 = skip")
    ap.add_argument("--no-extra", action="store_true", help="skip the secondary C3 (zstd) measurement")
    ap.add_argument("--extra-pages", type=int, default=1 << 20, help="pages for the C3 zstd measurement")
    ap.add_argument("--extra-steps", type=int, default=2)
    ap.add_argument("--config", default="C2", choices=["C2", "C4"],
                    help="C2: the headline (LZ4 compress+decompress, 1M x 16 KiB per GPU); "
                         "C4: BASELINE configs[3], LZ4 decompress-only of 8M x 8 KiB pages split over the ranks")
    ap.add_argument("--c4-pages", type=int, default=8 << 20, help="C4 total pages over all ranks")
    return ap.parse_args()


def host_cpu() -> tuple[int, str]:
    """(cores this process can run on, CPU model name): the affinity mask, capped by the cgroup CPU
    quota when one is set (the GPU box grants 16 CPUs of quota on a 256-CPU affinity mask; more
    threads than the quota only time-slice the same 16 CPUs)."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            cores = max(1, min(cores, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return cores, model


def cpu_baseline(codec: str, n: int, page_len: int, threads: int, seed: int, reps: int = 3) -> dict:
    """The reference's vendored codec on the host: oracle/_ref/cpu_baseline (C, pthreads by page range,
    one codec call per page, one thread per core of the affinity mask, best of `reps`), over the first n
    pages of the same generator; None when the reference build is not present."""
    import subprocess

    exe = os.path.join(ROOT, "oracle", "_ref", "cpu_baseline")
    if not os.path.exists(exe):
        return None
    out = subprocess.run([exe, codec, str(n), str(page_len), str(threads), str(reps), str(seed)],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=600)
    if out.returncode != 0:
        raise SystemExit(f"CPU baseline failed: {out.stdout.decode()} {out.stderr.decode()}")
    r = json.loads(out.stdout.decode().strip().splitlines()[-1])
    _, model = host_cpu()
    calls = {"lz4": "LZ4_compress_default/LZ4_decompress_safe (vendored LZ4 1.7.5)",
             "zstd": "ZSTD_compress(level 1)/ZSTD_decompress (vendored zstd 1.1.2)",
             "zlib": "compress2(level 1)/uncompress (vendored zlib 1.2.8)"}[codec]
    return {"value": r["combined_gib_s"], "unit": "GiB/s", "cores": r["threads"], "kind": "reference",
            "sample": f"first {n} of the same pages ({n * page_len / GIB:.1f} GiB), {calls} from oracle/_ref, "
                      f"one call per page, C pthreads by page range on {r['threads']} threads ({model}), "
                      f"best of {reps}",
            "compress_gib_s": r["compress_gib_s"], "decompress_gib_s": r["decompress_gib_s"], "ratio": r["ratio"]}


def pages_equal(out, pages, rv, plen: int) -> bool:
    """Every page decoded to its full length and bit-exact, compared in 1 GiB slices (torch.equal
    over the whole tensors would take a 16 GiB temporary).  Runs after the timed region."""
    step = max(1, (1 << 30) // plen)
    ok = bool((rv == plen).all().item())
    for a in range(0, out.shape[0], step):
        ok = ok and torch.equal(out[a:a + step], pages[a:a + step])
    return ok


def measure_codec(cid: int, name: str, n: int, plen: int, steps: int, warmup: int, dev, seed: int, first: int,
                  dist: int) -> dict:
    """Device-resident compress+decompress of n resident pages with codec `cid` (HIP events on the stream)."""
    pages = codec.pagegen(n, plen, seed=seed, first=first, dist=dist, device=dev)
    slot = codec.slot_size(plen, cid)
    comp = torch.empty((n, slot), dtype=torch.uint8, device=dev)
    clen = torch.empty((n,), dtype=torch.int32, device=dev)
    out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
    rv = torch.empty((n,), dtype=torch.int32, device=dev)
    codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen)
    torch.cuda.synchronize()
    mx = int(clen.max().item())
    for _ in range(max(warmup, 1)):
        codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen)
        codec.decompress_pages(comp, clen, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx)
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record()
        codec.compress_pages(pages, compressor_id=cid, out=comp, out_len=clen)
        ev[k][1].record()
        codec.decompress_pages(comp, clen, plen, compressor_id=cid, out=out, rv=rv, max_comp_len=mx)
        ev[k][2].record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # the last timed step's output, after the timed region
    if not (bool((clen > 0).all().item()) and pages_equal(out, pages, rv, plen)):
        raise SystemExit(f"{name}: round trip failed on the benchmark pages")
    c_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / steps
    d_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / steps
    nbytes = n * plen
    cbytes = int(clen.to(torch.int64).sum().item())
    algo = nbytes + cbytes
    res = {"pages": n, "page_len": plen, "steps": steps, "ms_per_step": round(wall / steps * 1e3, 3),
           "value": round(nbytes * steps / wall / GIB, 3), "unit": "GiB/s",
           "compress_gib_s": round(nbytes / (c_ms * 1e-3) / GIB, 3),
           "decompress_gib_s": round(nbytes / (d_ms * 1e-3) / GIB, 3),
           "kernel_ms": {f"{name}_encode": round(c_ms, 3), f"{name}_decode": round(d_ms, 3)},
           "roofline_by_kernel": {f"{name}_encode": round(algo / (c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                  f"{name}_decode": round(algo / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
           "algorithmic_bytes_per_launch": algo, "ratio": round(nbytes / cbytes, 4)}
    tr = {k: pmc_traffic(k, n, plen) for k in res["kernel_ms"]}
    res["traffic"] = {k: (v["bytes"] if v else None) for k, v in tr.items()}
    res["traffic_source"] = {k: ((v.get("source") or ("stale: " + v["stale"])) if v else None) for k, v in tr.items()}
    return res, pages


def e2e_host(pages_dev: torch.Tensor, n: int) -> dict:
    """PCIe-inclusive rate through the host batch API (malloc'd pages -> pinned -> H2D -> kernels -> D2H)."""
    import ctypes

    import numpy as np

    lib = _lib.load()
    host = pages_dev[:n].cpu().numpy()
    plen = host.shape[1]
    cap = codec.compress_bound(plen)
    comp = np.zeros((n, cap), dtype=np.uint8)
    out = np.zeros_like(host)
    # written once before the timed calls, as tyche's own buffers are (malloc + fill): calloc'd zero
    # pages would make the first call's scatter fault on every page (tools/host_probe.py does the same)
    comp.fill(1)
    out.fill(1)
    res = np.zeros(n, dtype=np.int32)
    rv = np.zeros(n, dtype=np.int32)
    vp = ctypes.c_void_p * n
    src_p = vp(*[host.ctypes.data + i * plen for i in range(n)])
    comp_p = vp(*[comp.ctypes.data + i * cap for i in range(n)])
    out_p = vp(*[out.ctypes.data + i * plen for i in range(n)])
    u32 = ctypes.c_uint32 * n
    slen = u32(*([plen] * n))
    ccap = u32(*([cap] * n))
    i32p = ctypes.POINTER(ctypes.c_int32)
    prof = (ctypes.c_uint64 * 8)()

    def stage_clocks():   # the engine's host-stage clocks since the last read (tyche_host_profile)
        lib.tyche_host_profile(prof, 8)
        return [int(x) for x in prof]
    reps = 3
    best_c = best_d = float("inf")
    acc = {"compress": [0] * 8, "decompress": [0] * 8}
    stage_clocks()
    for _ in range(reps):
        t0 = time.perf_counter()
        _lib.check(lib.tyche_compress_host(1, 1, n, src_p, slen, comp_p, ccap, res.ctypes.data_as(i32p)),
                   "tyche_compress_host")
        t1 = time.perf_counter()
        acc["compress"] = [a + b for a, b in zip(acc["compress"], stage_clocks())]
        clen = u32(*[int(x) for x in res])
        _lib.check(lib.tyche_decompress_host(1, n, comp_p, clen, out_p, slen, rv.ctypes.data_as(i32p)),
                   "tyche_decompress_host")
        t2 = time.perf_counter()
        acc["decompress"] = [a + b for a, b in zip(acc["decompress"], stage_clocks())]
        best_c, best_d = min(best_c, t1 - t0), min(best_d, t2 - t1)
    assert (rv == plen).all() and np.array_equal(out, host), "host-path round trip failed"
    nbytes = n * plen
    res = {"pages": n, "compress_gib_s": round(nbytes / best_c / GIB, 3),
           "decompress_gib_s": round(nbytes / best_d / GIB, 3),
           "combined_gib_s": round(nbytes / (best_c + best_d) / GIB, 3),
           "wall_ms": {"compress": round(best_c * 1e3, 3), "decompress": round(best_d * 1e3, 3)}}
    # where a call's time goes (engine.hip run_host_batch), ms per call averaged over the reps and summed
    # over the threads that ran each stage: waiting for a slot's stream (H2D + kernel + D2H not yet
    # overlapped), scattering results into the callers' buffers, gathering inputs into pinned memory,
    # enqueuing copies and kernels; plus the bytes gathered / scattered and the chunks per call
    res["stages_ms_per_call"] = {
        d: {"wait": round(v[0] / reps / 1e6, 3), "scatter": round(v[1] / reps / 1e6, 3),
            "gather": round(v[2] / reps / 1e6, 3), "enqueue": round(v[3] / reps / 1e6, 3),
            "gather_mib": round(v[4] / reps / 2 ** 20, 2), "scatter_mib": round(v[5] / reps / 2 ** 20, 2),
            "chunks": round(v[6] / reps, 2)} for d, v in acc.items()}
    link = pcie_probe(pages_dev.device, nbytes)
    res["link_probe"] = link
    # the ceiling each direction could reach if only the link moved bytes: compress sends the pages
    # and brings back ~1/ratio of them, decompress the reverse (both directions run at once)
    ratio = nbytes / float(sum(int(x) for x in clen))
    h2d, d2h = link["h2d_gib_s"], link["d2h_gib_s"]
    res["link_bound_compress_gib_s"] = round(min(h2d, d2h * ratio), 3)
    res["link_bound_decompress_gib_s"] = round(min(d2h, h2d * ratio), 3)
    res["frac_of_link_bound"] = {"compress": round(res["compress_gib_s"] / res["link_bound_compress_gib_s"], 3),
                                 "decompress": round(res["decompress_gib_s"] / res["link_bound_decompress_gib_s"], 3)}
    # the same with the smaller direction's bytes moving at the probe's bidirectional rate (both
    # directions at once) and the rest of the larger direction alone at its own rate
    bi = link["bidir_each_gib_s"]

    def both_ways(big, small, rate_big):   # GiB/s of uncompressed pages for `big` and `small` bytes
        t = small / bi + (big - small) / rate_big
        return nbytes / GIB / t
    comp_b = nbytes / ratio
    res["link_bound_bidir_gib_s"] = {"compress": round(both_ways(nbytes / GIB, comp_b / GIB, h2d), 3),
                                     "decompress": round(both_ways(nbytes / GIB, comp_b / GIB, d2h), 3)}
    res["frac_of_bidir_bound"] = {k: round(res[f"{k}_gib_s"] / v, 3) for k, v in res["link_bound_bidir_gib_s"].items()}
    return res


def pcie_probe(dev, nbytes: int, reps: int = 5) -> dict:
    """Raw pinned-host <-> HBM copy rates (hipMemcpyAsync through torch, 64 MiB copies back to back on one
    stream per direction, best of `reps`): the PCIe ceiling for the host path."""
    chunk = 64 << 20
    k = max(1, nbytes // chunk)
    h = [torch.empty(chunk, dtype=torch.uint8).pin_memory() for _ in range(2)]
    d = [torch.empty(chunk, dtype=torch.uint8, device=dev) for _ in range(2)]
    s_up, s_dn = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn):
        best = float("inf")
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return k * chunk / best / GIB

    def up():
        with torch.cuda.stream(s_up):
            for i in range(k):
                d[0].copy_(h[0], non_blocking=True)

    def down():
        with torch.cuda.stream(s_dn):
            for i in range(k):
                h[1].copy_(d[1], non_blocking=True)

    def both():
        up()
        down()
    return {"h2d_gib_s": round(timed(up), 3), "d2h_gib_s": round(timed(down), 3),
            "bidir_each_gib_s": round(timed(both), 3), "bytes_per_direction": k * chunk}


def pmc_traffic(kernel: str, pages: int, page_len: int):
    """HBM bytes per launch for `kernel` from the newest committed PMC summary
    (profiles/rNN_traffic*.json, made by tools/pmc_traffic.py from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes of the same kernels), scaled from bytes per page to this
    launch's page count.  A summary counts only if it was taken on the kernel sources this
    process runs (its kernel_sources_sha16 equals _build.kernel_sources_digest()); otherwise
    the result is None bytes with the stale file named, never a number from other code."""
    from tyche_amd._build import kernel_sources_digest
    cur = kernel_sources_digest()
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*_traffic*.json")))
    for f in reversed(files):
        t = json.load(open(f))
        if t.get("page_len") == page_len and kernel in t.get("bytes_per_page", {}):
            if t.get("kernel_sources_sha16") != cur:
                return {"bytes": None, "source": None, "stale": os.path.basename(f)}
            return {"bytes": int(t["bytes_per_page"][kernel] * pages), "source": os.path.basename(f),
                    "commit": t.get("commit")}
    return None


def run_c4(args, info, dev):
    """BASELINE configs[3]: LZ4 decompress-only (the restore path) of 8M x 8 KiB pages split across the ranks
    by contiguous page ranges (sharding.page_range, strong scaling: the total is fixed).  Each rank compresses
    its range once (untimed, every page round-trip checked), then times decode-only steps."""
    from tyche_amd import sharding

    plen = 8192
    a, n = sharding.page_range(args.c4_pages, info.rank, info.world)
    pages = codec.pagegen(n, plen, seed=args.seed, first=a, dist=args.dist, device=dev)
    comp, clen = codec.compress_pages(pages)
    torch.cuda.synchronize()
    mx = int(clen.max().item())
    out = torch.empty_like(pages)
    rv = torch.empty((n,), dtype=torch.int32, device=dev)
    for _ in range(max(args.warmup, 1)):
        codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=mx)
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    runner.barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        events[k][0].record()
        codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=mx)
        events[k][1].record()
    torch.cuda.synchronize()
    runner.barrier(info)
    elapsed = runner.max_over_ranks(info, time.perf_counter() - t0)
    if not pages_equal(out, pages, rv, plen):   # the last timed step's output, after the timed region
        raise SystemExit("C4: round trip failed")
    del pages
    comp_bytes = int(clen.to(torch.int64).sum().item())
    d_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    total = runner.sum_over_ranks(info, float(n))
    algo = n * plen + comp_bytes
    achieved = algo / (d_ms * 1e-3) / 1e9
    traffic = pmc_traffic("lz4_decode", n, plen)
    result = {
        "metric": "GiB/s device-resident LZ4 decompress, 8M x 8 KiB pages split over the GPUs (BASELINE configs[3])",
        "value": round(total * plen * args.steps / elapsed / GIB, 3), "unit": "GiB/s", "n_gpus": info.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (pagegen.h PostgreSQL-like pages, seed 20170303)",
        "config": {"workload": "C4: LZ4 decompress-only, 8M x 8 KiB pages, contiguous page ranges per rank",
                   "total_pages": args.c4_pages, "pages_this_rank": n, "page_len": plen, "codec": "lz4",
                   "parallelism": f"page-range x{info.world}"},
        "roofline": {"bound": "hbm", "kernel": "lz4_decode", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic["bytes"] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None,
                     "traffic_stale": traffic.get("stale") if traffic else None,
                     "algorithmic_bytes_per_launch": algo},
        "kernel_ms": {"lz4_decode": round(d_ms, 4)}, "ratio": round(n * plen / comp_bytes, 4),
    }
    if info.rank == 0:
        print(json.dumps(result), flush=True)
    runner.shutdown(info)


def main():
    args = parse()
    info = runner.init_distributed()
    if args.config == "C4":
        dev = torch.device("cuda", info.local_rank)
        torch.cuda.set_device(dev)
        if _lib.load().tyche_device_ready() != 1:
            raise SystemExit(f"device not ready: {_lib.last_error()}")
        return run_c4(args, info, dev)
    dev = torch.device("cuda", info.local_rank)
    torch.cuda.set_device(dev)
    lib = _lib.load()
    if lib.tyche_device_ready() != 1:
        raise SystemExit(f"device not ready: {_lib.last_error()}")

    n, plen = args.pages, args.page_len
    first = info.rank * n                       # weak scaling: each rank owns its own 1M pages
    pages = codec.pagegen(n, plen, seed=args.seed, first=first, dist=args.dist, device=dev)
    slot = codec.slot_size(plen)
    comp = torch.empty((n, slot), dtype=torch.uint8, device=dev)
    clen = torch.empty((n,), dtype=torch.int32, device=dev)
    out = torch.empty((n, plen), dtype=torch.uint8, device=dev)
    rv = torch.empty((n,), dtype=torch.int32, device=dev)

    def step(ev=None, max_comp=0):
        if ev is not None:
            ev[0].record()
        codec.compress_pages(pages, out=comp, out_len=clen)
        if ev is not None:
            ev[1].record()
        codec.decompress_pages(comp, clen, plen, out=out, rv=rv, max_comp_len=max_comp)
        if ev is not None:
            ev[2].record()

    # warm-up (the timed steps' output is checked after the timed region: every page round-trips
    # bit-exactly)
    step()
    torch.cuda.synchronize()
    max_comp = int(clen.max().item())
    for _ in range(max(args.warmup - 1, 0)):
        step(max_comp=max_comp)
    # no other kernel between the warm-up and the timed steps: the first LZ4 decode after a foreign
    # kernel on the stream (a torch reduction, fill or compare) ran 29.3 instead of 23.8 ms on every
    # box tried (profiles/r06_steps*.jsonl); the byte count and the check come after the timed region
    torch.cuda.synchronize()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    runner.barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k], max_comp)
    torch.cuda.synchronize()
    runner.barrier(info)
    t1 = time.perf_counter()
    elapsed = runner.max_over_ranks(info, t1 - t0)
    if not (bool((clen > 0).all().item()) and pages_equal(out, pages, rv, plen)):
        raise SystemExit("round trip failed on the benchmark pages")
    comp_bytes = int(clen.to(torch.int64).sum().item())

    c_ms = sum(e[0].elapsed_time(e[1]) for e in events) / args.steps
    d_ms = sum(e[1].elapsed_time(e[2]) for e in events) / args.steps
    page_bytes = n * plen
    total_pages = runner.sum_over_ranks(info, float(n))
    value = total_pages * plen * args.steps / elapsed / GIB
    algo_bytes = page_bytes + comp_bytes            # per launch, either direction
    kernels = {"lz4_encode": c_ms, "lz4_decode": d_ms}
    dom = max(kernels, key=kernels.get)
    achieved = algo_bytes / (kernels[dom] * 1e-3) / 1e9
    traffic = pmc_traffic(dom, n, plen)

    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (pagegen.h PostgreSQL-like heap/index pages, LZ4 ratio ~2.65, seed 20170303)",
        "config": {"workload": "C2: LZ4 block compress+decompress, 1M x 16 KiB pages per GPU, device-resident",
                   "pages_per_gpu": n, "page_len": plen, "codec": "lz4", "parallelism": f"page-range x{info.world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic["bytes"] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None,
                     "traffic_commit": traffic.get("commit") if traffic else None,
                     "traffic_stale": traffic.get("stale") if traffic else None,
                     "algorithmic_bytes_per_launch": algo_bytes},
        "compress_gib_s": round(page_bytes / (c_ms * 1e-3) / GIB, 3),
        "decompress_gib_s": round(page_bytes / (d_ms * 1e-3) / GIB, 3),
        "kernel_ms": {"lz4_encode": round(c_ms, 4), "lz4_decode": round(d_ms, 4)},
        "kernel_ms_steps": {"lz4_encode": [round(e[0].elapsed_time(e[1]), 3) for e in events],
                            "lz4_decode": [round(e[1].elapsed_time(e[2]), 3) for e in events]},
        "roofline_by_kernel": {k: round(algo_bytes / (v * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for k, v in kernels.items()},
        "ratio": round(page_bytes / comp_bytes, 4),
    }
    if info.rank == 0 and info.world == 1:
        threads = args.cpu_threads or host_cpu()[0]
        if args.e2e_pages > 0:
            result["e2e_host_path"] = e2e_host(pages, min(args.e2e_pages, n))
        if not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline("lz4", min(max(args.cpu_pages, threads * 2048), n), plen, threads,
                                                  args.seed)
        if not args.no_extra:
            # C3 (configs[2]): zstd level-1 compress+decompress, 1M x 32 KiB pages, 1 GPU -- reported
            # beside the headline line, never as `value`
            del pages, comp, clen, out, rv
            torch.cuda.empty_cache()
            c3, zpages = measure_codec(3, "zstd", args.extra_pages, 32768, args.extra_steps, 1, dev, args.seed, 0,
                                       args.dist)
            c3["workload"] = "C3: zstd level-1 compress+decompress, 1M x 32 KiB pages, 1 GPU, device-resident"
            if not args.no_cpu:
                c3["cpu_baseline"] = cpu_baseline("zstd", min(max(32768, threads * 256), args.extra_pages), 32768,
                                                  threads, args.seed, reps=2)
            result["configs"] = {"C3_zstd": c3}
            del zpages
            torch.cuda.empty_cache()
            # C4 (configs[3]) per GPU: LZ4 decompress of 8M x 8 KiB pages over 8 GPUs is 1M x 8 KiB
            # pages on each (page-range shards, no collective); its one-GPU shard, decode rate reported
            c4, c4pages = measure_codec(1, "lz4", args.extra_pages, 8192, max(args.extra_steps, 3), 1, dev,
                                        args.seed, 0, args.dist)
            c4["workload"] = ("C4 shard: LZ4 compress+decompress of 1M x 8 KiB pages on one GPU (C4 = 8M pages "
                              "over 8 GPUs, decompress_gib_s is its per-GPU rate)")
            result["configs"]["C4_lz4_8k_shard"] = c4
            del c4pages
            torch.cuda.empty_cache()
    if info.rank == 0:
        print(json.dumps(result), flush=True)
    runner.shutdown(info)


if __name__ == "__main__":
    main()
