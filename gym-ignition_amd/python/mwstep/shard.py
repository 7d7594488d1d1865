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


def gather_obs(obs, group=None):
    """All-gather equal-sized per-rank observation slabs [W_local, n_obs] into
    [W_local * world_size, n_obs], rank-major (global world order)."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo" and obs.is_cuda:
        # gloo (CPU rehearsal of a multi-rank run) gathers host copies
        return gather_obs(obs.cpu(), group).to(obs.device)
    out = torch.empty((ws * obs.shape[0],) + tuple(obs.shape[1:]), dtype=obs.dtype, device=obs.device)
    dist.all_gather_into_tensor(out, obs.contiguous(), group=group)
    return out
