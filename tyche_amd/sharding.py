"""Per-rank page partitioning.

Pages are independent (no cross-page state in any codec: noDict, lz4.c:667;
fresh contexts per call), so N GPUs each take a contiguous page range and
no data-path collective is needed.  The only cross-rank traffic is the
barrier and the max-over-ranks timing reduction that bench.py performs.
"""
from __future__ import annotations


def page_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """[first, first+count) of a contiguous split of `total` pages; sizes differ by at most one."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return first, count


def weak_range(per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: every rank owns `per_rank` pages, rank r's are [r*per_rank, (r+1)*per_rank)."""
    return rank * per_rank, per_rank
