"""One process per GPU: batch sharding and the single RCCL exchange of BER accounting.

Decoding shards embarrassingly: rank r of W decodes the contiguous codewords
[offset, offset + count) of the global batch, with its channel noise drawn at the global codeword
index (nldpc.channel.awgn_llr b_offset), so the union of the shards is the single-GPU decode of the
whole batch.  The only collective is after decoding: a SUM all_reduce of the int64 [T, 2] error
counters (about 320 bytes per rank over xGMI) and a MAX all_reduce of the timed region.
Backend "nccl" is RCCL on ROCm; the helpers are backend-agnostic (gloo in the CPU tests).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl"):
    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard(total: int, rank: int, world: int):
    """Contiguous shard (offset, count) of `total` codewords for `rank`; remainders go to the low ranks."""
    base, rem = divmod(total, world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def _all_reduce(t: torch.Tensor, op) -> torch.Tensor:
    """all_reduce in place; device tensors go through host memory when the backend is gloo (the CPU
    test backend, also used by the GPU test whose two ranks share one GPU)."""
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)
    return t


def sum_counts(counts: torch.Tensor) -> torch.Tensor:
    """All-reduce (SUM) the per-iteration (bit errors, frame errors) counters in place."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        _all_reduce(counts, dist.ReduceOp.SUM)
    return counts


def max_time(seconds: float, device=None) -> float:
    """The job's time for a region: the maximum over ranks."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    _all_reduce(t, dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device_index=None):
    if dist.is_initialized() and dist.get_world_size() > 1:
        if device_index is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device_index])
        else:
            dist.barrier()


def finalize():
    if dist.is_initialized():
        dist.destroy_process_group()
