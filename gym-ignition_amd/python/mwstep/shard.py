"""Sharding of worlds over ranks (one process per GPU).

Worlds are independent, so a rank simply owns a contiguous block of global
world indices; its Philox reset streams are keyed by the GLOBAL index
(``world_offset``), which makes every world's trajectory independent of the
number of GPUs.  The only collective is the optional all-gather of the final
observation tensor (RCCL over xGMI with the "nccl" backend, gloo on CPU).
"""

from typing import Tuple


def shard_range(n_global: int, rank: int, world_size: int) -> Tuple[int, int]:
    """[begin, end) of the global worlds owned by `rank` (contiguous blocks,
    the first n_global % world_size ranks get one extra world)."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    q, r = divmod(n_global, world_size)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def gather_obs(obs, group=None, n_global=None):
    """All-gather the per-rank observation slabs [W_local, n_obs] into
    [W_global, n_obs], rank-major (global world order).  Slabs may differ by
    one world (shard_range of a world count the ranks do not divide): each
    rank pads its slab to the largest one, one all_gather_into_tensor moves
    the padded slabs, the padding is dropped.  Slab sizes come from
    shard_range(n_global, ...) when n_global is given, else from a first
    all-gather of the sizes."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo" and obs.is_cuda:
        # gloo (CPU rehearsal of a multi-rank run) gathers host copies
        return gather_obs(obs.cpu(), group, n_global).to(obs.device)
    if n_global is not None:
        sizes = [e - b for b, e in (shard_range(n_global, r, ws) for r in range(ws))]
        if sizes[dist.get_rank(group)] != obs.shape[0]:
            raise ValueError(f"slab of {obs.shape[0]} worlds, shard_range({n_global}) expects "
                             f"{sizes[dist.get_rank(group)]}")
    else:
        mine = torch.tensor([obs.shape[0]], dtype=torch.int64, device=obs.device)
        every = torch.empty(ws, dtype=torch.int64, device=obs.device)
        dist.all_gather_into_tensor(every, mine, group=group)
        sizes = [int(v) for v in every.tolist()]
    m = max(sizes)
    slab = obs.contiguous()
    if obs.shape[0] < m:
        slab = torch.cat([slab, slab.new_zeros((m - obs.shape[0],) + tuple(obs.shape[1:]))])
    out = torch.empty((ws * m,) + tuple(obs.shape[1:]), dtype=obs.dtype, device=obs.device)
    dist.all_gather_into_tensor(out, slab, group=group)
    if all(sz == m for sz in sizes):
        return out
    return torch.cat([out[r * m:r * m + sz] for r, sz in enumerate(sizes)])
