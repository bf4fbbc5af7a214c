"""Data-parallel sharding of explanation work over ranks (one process per GPU).

Target events are independent given the replicated read-only graph, feature tables and weights, and
every random draw is keyed by the GLOBAL event id (include/tempme.h RNG contract), so a rank's
results do not depend on which other events share its batch or its GPU: sharding needs no
data-path collective. Ranks process whole reference batches (the attention std of
explainer_new.py:828 is batch-global), and only the benchmark's barrier and max-over-ranks timing
touch the process group.
"""
import numpy as np


def shard_events(step, rank, world, per_rank, n_events):
    """Rank ``rank``'s events at ``step``: (row indices into the event list, cycling; keyed event ids).

    Consecutive ranks take consecutive blocks of ``per_rank`` events, steps follow each other, so the
    union over ranks of one step is one contiguous block of global event ids."""
    if not (0 <= rank < world) or per_rank < 0 or n_events <= 0:
        raise ValueError("shard_events: bad rank/world/per_rank/n_events")
    first = (int(step) * world + rank) * per_rank
    gid = np.arange(first, first + per_rank, dtype=np.int64)
    return gid % n_events, gid.astype(np.uint32)


def max_over_ranks(value, dist=None, device="cpu"):
    """Max of a per-rank float over the process group (identity without one)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
