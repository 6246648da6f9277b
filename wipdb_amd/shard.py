"""Multi-GPU sharding of the batch: blocks are independent, so
the work is split into contiguous ranges with NO data-path collective.

* ``block_shard``       weak scaling of the headline bench: rank r owns its own
                        fixed-size range of blocks [r*B, (r+1)*B).
* ``byte_balanced_cuts`` contiguous span ranges balanced by bytes (mixed
                        sizes), the rule hcrc_batch_multi applies in C++
                        (wipdb_amd/csrc/hcrc_api.cc): weight = length + 64.
* ``max_over_ranks``    the timing reduction of the bench contract (the only
                        cross-rank communication; never on the data path).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

SPAN_OVERHEAD = 64  # per-span weight added to its length (descriptor + fold cost)


def block_shard(rank: int, world: int, blocks_per_rank: int) -> Tuple[int, int]:
    """(first_block, count) of rank's shard under weak scaling."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} not in [0, {world})")
    return rank * blocks_per_rank, blocks_per_rank


def byte_balanced_cuts(lengths, world: int) -> List[int]:
    """cut[k]..cut[k+1] = span range of shard k (len world+1), contiguous and
    balanced by length + 64 -- identical to hcrc_batch_multi's split."""
    if world <= 0:
        raise ValueError("world must be positive")
    w = np.asarray(lengths, dtype=np.uint64) + np.uint64(SPAN_OVERHEAD)
    count = int(w.size)
    cut = [0] + [count] * world
    if count == 0:
        return cut
    total = int(w.sum())
    acc = np.cumsum(w, dtype=np.uint64)
    # smallest i+1 with acc[i] >= total*d/world (integer division as in C++)
    for d in range(1, world):
        thr = np.uint64(total * d // world)
        cut[d] = int(np.searchsorted(acc, thr, side="left")) + 1
        cut[d] = min(cut[d], count)
    for d in range(1, world + 1):  # monotone, as the C++ loop produces
        cut[d] = max(cut[d], cut[d - 1])
    return cut


def max_over_ranks(x: float, device=None) -> float:
    """MAX of a per-rank float over the default process group (identity when
    torch.distributed is not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
