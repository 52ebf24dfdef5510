"""Env-batch sharding across GPUs.

Environments are independent: a global batch of envs is split into
contiguous per-rank blocks and every rank steps its block on its own GPU.
There is no data-path collective; ranks only meet for barriers and the
max-over-ranks timing reduction.  RNG streams (scan noise, autoreset spawns)
are keyed by *global* env id (f110_config.env_offset), so an env's
trajectory does not depend on how many GPUs share the batch.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    offset: int   # global id of this rank's first env
    count: int    # envs on this rank


def shard_range(total: int, world: int, rank: int) -> Shard:
    """Contiguous near-equal blocks: the first total % world ranks get one more."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, extra = divmod(int(total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return Shard(rank, world, offset, count)


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def local_device_index(local_rank: int) -> int:
    """GPU of this rank: LOCAL_RANK (one process per GPU).  F110_SAME_DEVICE=1
    maps every rank to GPU 0 (rehearsing the multi-rank path on a 1-GPU box)."""
    if os.environ.get("F110_SAME_DEVICE") == "1":
        return 0
    n = torch.cuda.device_count()  # counts devices without initialising HIP
    if local_rank >= n:
        raise RuntimeError(f"LOCAL_RANK {local_rank} but {n} visible GPU(s): one rank per GPU "
                           "(F110_SAME_DEVICE=1 rehearses several ranks on GPU 0)")
    return local_rank


def init(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from torchrun's env (no-op for world 1)."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or os.environ.get("F110_DIST_BACKEND")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local_device_index(local))
            kw["device_id"] = torch.device(f"cuda:{local_device_index(local)}")
        dist.init_process_group(backend=backend, **kw)
        self_check()
    return rank, world, local


def self_check() -> None:
    """One all-reduce of (rank + 1) on the backend's own device: every rank must
    see 1 + 2 + ... + world.  A broken collective path (RCCL over xGMI, or a
    rank on the wrong device) fails here, loudly, before any timed work."""
    world = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(dist.get_rank() + 1)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    want = world * (world + 1) / 2.0
    if float(t.item()) != want:
        raise RuntimeError(f"torch.distributed self-check failed: all-reduce gave {float(t.item())}, want {want} "
                           f"(backend {dist.get_backend()}, rank {dist.get_rank()} of {world})")


def describe() -> dict:
    """What the ranks run on: torch.distributed's backend (None for one
    process) and world size, for the bench line's config."""
    if dist.is_available() and dist.is_initialized():
        return {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(),
                "same_device": os.environ.get("F110_SAME_DEVICE") == "1"}
    return {"backend": None, "world_size": 1, "same_device": False}


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def max_over_ranks(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def sum_tensor_over_ranks(t: torch.Tensor) -> torch.Tensor:
    """Element-wise sum of an int64 / float64 CPU tensor over the ranks (a
    copy; the input itself when there is one rank)."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    x = t.to(dev).clone()
    dist.all_reduce(x, op=dist.ReduceOp.SUM)
    return x.cpu()


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
