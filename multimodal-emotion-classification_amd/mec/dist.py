"""Sample-sharded data parallelism for the tri-modal path.

One process per GPU. A global batch is cut into contiguous per-rank shards; every rank
runs all three encoders AND the fusion step on its own shard (no feature exchange), then
one all-gather collects the 34-float result rows (3x7 modality probs, 7 fused probs,
3 attention weights, 3 decision weights). With backend "nccl" (= RCCL on ROCm) the
all-gather runs over xGMI; "gloo" is used for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

ROW = 34


def shard(total: int, world: int, rank: int):
    """Contiguous, balanced [start, stop) of `total` samples for `rank`."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def all_gather_rows(rows: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """Gather per-rank [n_r, ROW] shards (n_r from shard()) into the global [total, ROW]."""
    world = dist.get_world_size(group)
    cap = -(-total // world)
    if rows.shape[0] > cap:
        raise ValueError('shard larger than ceil(total/world)')
    padded = rows
    if rows.shape[0] < cap:
        padded = torch.zeros((cap, rows.shape[1]), dtype=rows.dtype, device=rows.device)
        padded[:rows.shape[0]] = rows
    if dist.get_backend(group) == 'nccl':
        out = torch.empty((world * cap, rows.shape[1]), dtype=rows.dtype, device=rows.device)
        dist.all_gather_into_tensor(out, padded.contiguous(), group=group)
        parts = list(out.split(cap))
    else:
        parts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(parts, padded.contiguous(), group=group)
    pieces = []
    for r in range(world):
        a, b = shard(total, world, r)
        pieces.append(parts[r][:b - a])
    return torch.cat(pieces, dim=0)


def pack_rows(s_probs, t_probs, i_probs, f_probs, attn_w, dec_w) -> torch.Tensor:
    return torch.cat([s_probs, t_probs, i_probs, f_probs, attn_w, dec_w], dim=1)
