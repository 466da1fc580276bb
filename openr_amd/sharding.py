"""Source sharding across GPUs.

Every SPF source (and every what-if (source, link) pair) is independent given
the read-only topology, so the all-sources sweep shards with no data-path
collective: each rank replicates the CSR mirror and runs a contiguous block
of the name-ordered source list. Only the bench timing (barrier, max over
ranks) and optional result checksums cross ranks.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of n units for `rank`; blocks differ in size
    by at most one and cover 0..n-1 exactly once."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_sources(sources: Sequence[str], world: int, rank: int) -> List[str]:
    lo, hi = shard_bounds(len(sources), world, rank)
    return list(sources[lo:hi])


def dist_env():
    """(rank, world_size, local_rank) from torch.distributed.run's env."""
    import os
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))
