"""Multi-GPU distribution of independent DoRC2DGI() frames.

At the reference's sizes the GI path has no exchange step: every frame (scene) is
independent, so N GPUs run N replicas -- or a batch of scenes dealt round-robin to the
ranks (BASELINE.json configs[4]: 64 x 4096^2 scenes, one scene per stream, 8 GPUs).  No
data-path collective exists; the only cross-rank traffic is the barrier and the
max-over-ranks timing reduction of the benchmark.

One process per GPU, launched by torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT from the environment); backend "nccl" (= RCCL) on the GPU box,
"gloo" in CPU tests.
"""
from __future__ import annotations

import os
from typing import List, Sequence


def env_ranks():
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str = "nccl"):
    """Initialise the process group when WORLD_SIZE > 1; returns (rank, local_rank, world)."""
    import torch
    import torch.distributed as dist

    rank, local, world = env_ranks()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, local, world


def shard(n_items: int, rank: int, world: int) -> List[int]:
    """Round-robin deal of item ids to ranks (scene s -> rank s % world)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return list(range(rank, n_items, world))


def scene_seed(item: int, base: int = 1000) -> int:
    """Deterministic scene seed for batch item `item` (independent of the rank count)."""
    return base + item


def max_over_ranks(values: Sequence[float], device: str = "cpu") -> List[float]:
    """Element-wise max over ranks (the benchmark's max-over-ranks timing)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def barrier() -> None:
    import torch.distributed as dist

    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
