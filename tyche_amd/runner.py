"""Process-group plumbing for multi-GPU runs (one process per GPU).

Pages shard by contiguous range, so the data path has no collective.  The only
cross-rank operations are the start/stop barrier and the max-over-ranks
reduction of the timed interval that bench.py reports (RCCL on GPUs, gloo on
CPU for the tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class RankInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = ""


def init_distributed(prefer_nccl: bool = True) -> RankInfo:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return RankInfo(rank=0, world=1, local_rank=0, backend="")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = "nccl" if (prefer_nccl and torch.cuda.is_available()) else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return RankInfo(rank=rank, world=world, local_rank=local, backend=backend)


def _device_for(info: RankInfo) -> torch.device:
    return torch.device("cuda", info.local_rank) if info.backend == "nccl" else torch.device("cpu")


def barrier(info: RankInfo) -> None:
    if info.world > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def max_over_ranks(info: RankInfo, value: float) -> float:
    if info.world <= 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_device_for(info))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(info: RankInfo, value: float) -> float:
    if info.world <= 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_device_for(info))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def shutdown(info: RankInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()
