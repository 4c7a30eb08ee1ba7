"""Multi-rank plumbing on CPU (gloo, world_size 2): page-range sharding with no
data-path collective, the start/stop barrier and the max-over-ranks timing that
bench.py reports.  Each rank checks its own shard with the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tyche_amd.sharding import page_range, weak_range


def test_page_range_partitions():
    for total in (0, 1, 7, 64, 1000, 1 << 20):
        for world in (1, 2, 3, 4, 8):
            spans = [page_range(total, r, world) for r in range(world)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for first, count in spans:
                assert first == pos
                pos += count
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    assert weak_range(1 << 20, 3) == (3 << 20, 1 << 20)
    with pytest.raises(ValueError):
        page_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, plen, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import time

    from oracle import oracle as O
    from tyche_amd import runner
    info = runner.init_distributed(prefer_nccl=False)
    assert info.backend == "gloo" and info.world == world
    first, count = page_range(total, info.rank, info.world)
    pages = O.pagegen(count, plen, seed=20170303, first=first, dist=0)
    runner.barrier(info)
    t0 = time.perf_counter()
    comp_bytes = 0
    for p in pages:
        c = O.lz4_compress(p.tobytes())
        r, out = O.lz4_decompress(c, plen)
        assert r == plen and out == p.tobytes()
        comp_bytes += len(c)
    runner.barrier(info)
    dt = time.perf_counter() - t0
    tmax = runner.max_over_ranks(info, dt)
    pages_all = runner.sum_over_ranks(info, float(count))
    q.put((info.rank, first, count, dt, tmax, pages_all, comp_bytes))
    runner.shutdown(info)


def test_gloo_two_ranks_shard_and_time():
    world, total, plen = 2, 41, 8192
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, plen, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == [0, 1]
    assert res[0][1] == 0 and res[0][1] + res[0][2] == res[1][1] and res[1][1] + res[1][2] == total
    tmax = res[0][4]
    assert tmax == res[1][4] and tmax >= max(r[3] for r in res) - 1e-9
    assert res[0][5] == total
    # the shards together are exactly the single-rank workload
    from oracle import oracle as O
    whole = O.pagegen(total, plen, seed=20170303, first=0, dist=0)
    assert sum(r[6] for r in res) == sum(len(O.lz4_compress(p.tobytes())) for p in whole)
    assert np.array_equal(O.pagegen(res[1][2], plen, first=res[1][1]), whole[res[1][1]:])
