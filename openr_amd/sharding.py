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


def weighted_blocks(weights: Sequence[float], world: int) -> List[Tuple[int, int]]:
    """Contiguous blocks [lo, hi) of units whose total weights are as equal as
    a contiguous split allows (prefix-sum cut points). Used for source shards
    weighted by per-source work, so high-degree nodes (Clos spines: many
    first-hop rows) spread over the ranks while every block stays a run of
    name-ordered sources (the multi-source BFS batches consecutive sources)."""
    n = len(weights)
    if world < 1:
        raise ValueError("world must be >= 1")
    total = float(sum(weights))
    cuts, acc, k = [0], 0.0, 1
    for i, w in enumerate(weights):
        acc += w
        while k < world and acc >= total * k / world and len(cuts) <= k:
            cuts.append(i + 1)
            k += 1
    while len(cuts) < world:
        cuts.append(n)
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def degree_weighted_sources(sources: Sequence[str], degrees: Sequence[int], world: int,
                            rank: int, per_neighbour: float = 1.0 / 16) -> List[str]:
    """Rank's contiguous block of `sources` with work weight 1 + deg/16 per
    source (degree-weighted sharding for Clos spines)."""
    lo, hi = weighted_blocks([1.0 + d * per_neighbour for d in degrees], world)[rank]
    return list(sources[lo:hi])


def dist_env():
    """(rank, world_size, local_rank) from torch.distributed.run's env."""
    import os
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def gather_source_tables(local_dist, local_nh, n_sources: int, group=None):
    """All-gather per-source tables for a central RIB.

    Rank r holds rows shard_bounds(n_sources, world, r) of the dist table
    (u32 [rows, N], viewed as int32) and of the first-hop table ([rows, N*W]).
    Blocks differ in size by at most one, so each rank pads its block to
    ceil(n_sources / world) rows and one all_gather_into_tensor per table
    moves everything (RCCL over xGMI on GPUs, gloo on CPU). Returns the full
    [n_sources, ...] tables on every rank, rows in source order.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(n_sources, world, rank)
    if local_dist.shape[0] != hi - lo or local_nh.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: expected {hi - lo} rows, got "
                         f"{local_dist.shape[0]} / {local_nh.shape[0]}")
    block = -(-n_sources // world)
    out = []
    for t in (local_dist, local_nh):
        padded = t.new_zeros((block,) + tuple(t.shape[1:]))
        padded[: hi - lo] = t
        full = t.new_empty((block * world,) + tuple(t.shape[1:]))
        dist.all_gather_into_tensor(full, padded, group=group)
        keep = torch.cat([full[r * block: r * block + (shard_bounds(n_sources, world, r)[1]
                                                        - shard_bounds(n_sources, world, r)[0])]
                          for r in range(world)])
        out.append(keep)
    return out[0], out[1]


def sharded_all_sources(ls_impl, sources: Sequence[str], use_link_metric: bool = True,
                        group=None):
    """All-sources SPF sharded over the ranks of `group`, gathered on every
    rank: each rank runs its contiguous block of `sources` on its own GPU (the
    CSR mirror is replicated), copies the rows into torch tensors and the
    tables are all-gathered. The mask width W is the whole batch's, so every
    rank's rows have the same shape. Returns (dist [S, N] int32 view of u32,
    nh [S, N*W] int32 view of u32, W) on the current CUDA device."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    words = ls_impl.spf_words(list(sources))
    mine = shard_sources(sources, world, rank)
    dev = torch.device("cuda", torch.cuda.current_device())
    sweep = ls_impl.sweep(mine, use_link_metric, words) if mine else None
    n = len(ls_impl.node_names())
    d = torch.empty((len(mine), n), dtype=torch.int32, device=dev)
    h = torch.empty((len(mine), n * words), dtype=torch.int32, device=dev)
    if sweep is not None:
        sweep.run()
        sweep.sync()
        sweep.copy_to(d.data_ptr(), h.data_ptr())
    if world == 1:
        return d, h, words
    full_d, full_h = gather_source_tables(d, h, len(sources), group)
    return full_d, full_h, words
