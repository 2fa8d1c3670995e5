"""Multi-GPU sharding: blocks and WAL log blocks are
independent, so a batch splits into contiguous ranges of the descriptor
array, one per rank (one process per GPU), sized by BYTES rather than count
so mixed block sizes balance.  No collective touches the data path; the
only cross-rank traffic is the timing barrier, a max over ranks of the
elapsed time and (optionally) a sum of per-rank counters (units processed,
mismatches).  Backend: "nccl" (RCCL) with a GPU, "gloo" on the CPU."""
import os

import numpy as np
import torch
import torch.distributed as dist


def setup(cpu_only=False):
    """(world, rank, local_rank) from the torch.distributed.run environment;
    initialises the process group when world > 1 (RCCL with a GPU, gloo on
    the CPU or when cpu_only: then no GPU call is made at all)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = not cpu_only and torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend="nccl" if gpu else "gloo")
    return world, rank, local


def _device():
    return "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([int(x)], dtype=torch.int64, device=_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def byte_ranges(sizes, world):
    """Contiguous [lo, hi) descriptor ranges, one per rank, with near-equal
    byte totals: rank r starts at the first block whose byte prefix reaches
    r/world of the total (a rank may get an empty range only if one block
    outweighs a whole share)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    n = len(sizes)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    prefix = np.concatenate([[0], np.cumsum(sizes)])
    total = int(prefix[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        cuts.append(int(np.searchsorted(prefix, target, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.asarray(cuts), n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def rank_slice(sizes, rank, world, trailer=5):
    """This rank's part of one described SST batch (blocks packed back to back,
    payload n_i + `trailer` bytes each): (lo, hi, first byte offset)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    lo, hi = byte_ranges(sizes, world)[rank]
    start = int(sizes[:lo].sum()) + trailer * lo
    return lo, hi, start


def local_shard(offsets, sizes, rank, world):
    """This rank's (offsets, sizes) slice of a batch (host or device arrays)."""
    lo, hi = byte_ranges(np.asarray(sizes.cpu() if torch.is_tensor(sizes) else sizes), world)[rank]
    return offsets[lo:hi], sizes[lo:hi], (lo, hi)
