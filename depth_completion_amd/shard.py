"""Frame sharding across GPUs of one node.

Frames never interact in the guided sampler (GroupNorm, loss, gradient rescale and Adam are all
per-frame; every call draws the same initial noise, marigold_dc.py:661, 677-684), so a sequence is
split into contiguous frame ranges, one per rank, with the weights replicated.  There is no
data-path collective: ranks exchange only their wall-clock time (max-over-ranks) for reporting.
Contiguous ranges keep predict.py's ``--use-prev-latent`` warm-start chain (predict.py:697-699)
inside each rank; it is broken only at the world-1 shard seams (each rank's first frame starts
from noise).
"""
from __future__ import annotations

import time
from typing import Callable, Sequence


def frame_shard(num_frames: int, rank: int, world: int) -> range:
    """Contiguous, balanced frame range of ``rank``: sizes differ by at most one, union = all frames."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(num_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def run_shard(fn: Callable, frames: Sequence, rank: int, world: int, batch: int = 1,
              use_prev_latent: bool = False, sync: Callable | None = None):
    """Run ``fn(frames[i:i+batch], prev_latents) -> (denses, latents)`` over this rank's shard.

    Returns ``(outputs, elapsed_s)`` where outputs is a list of (frame_index, dense, latent).  With
    ``use_prev_latent`` the previous call's latents seed the next call inside the shard (batch 1
    only, as in predict.py).
    """
    if use_prev_latent and batch != 1:
        raise ValueError("use_prev_latent requires batch 1 (predict.py:273-279)")
    idx = list(frame_shard(len(frames), rank, world))
    outs, prev = [], None
    t0 = time.perf_counter()
    for b in range(0, len(idx), batch):
        sel = idx[b:b + batch]
        dense, lat = fn([frames[i] for i in sel], prev if use_prev_latent else None)
        prev = lat
        for j, i in enumerate(sel):
            outs.append((i, dense[j], lat[j]))
    if sync is not None:
        sync()
    return outs, time.perf_counter() - t0


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host scalar over all ranks (timing only; no data-path exchange)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
