"""Row-sharded search across GPUs: one process per GPU, RCCL all-gather of top-k.

The reference has no multi-device path: it scans one process's Arrow chunks
(src/fenix/io/index/index.py:162) and selects over the concatenated table
(index.py:166; multi-source concat table.py:19-21).  Because
``topk(rows of all shards) == topk(concat of per-shard topk)`` for the
(distance, row) order, each rank scans its contiguous row range
``[row_base, row_base + n_local)`` with no data-path collective, and the only
exchange is one all-gather of ``nq * k`` (distance f32, row i64) pairs per
rank (1.2 KB at k=100) — latency-bound, so it is issued as a single
collective per query batch — followed by the deterministic merge kernel
(``fx_topk_merge``) on every rank.

With ``backend="nccl"`` (RCCL over xGMI on MI355X) tensors stay on the GPU;
with ``gloo`` (CPU tests) they are CPU tensors.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_rows(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous row range of ``rank``: (row_base, n_local), sizes differ by <= 1."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def allgather_topk(
    dist_t: torch.Tensor, row_t: torch.Tensor, group: Optional[dist.ProcessGroup] = None
) -> Tuple[torch.Tensor, torch.Tensor]:
    """[nq, k] per rank -> [nq, world, k] on every rank (one collective).

    Distances travel bit-cast to int64 beside the rows in a single [nq, k, 2]
    int64 buffer so one all-gather moves both.
    """
    world = dist.get_world_size(group)
    nq, k = dist_t.shape
    packed = torch.stack(
        [dist_t.contiguous().view(torch.int32).to(torch.int64), row_t.contiguous()], dim=-1
    )
    out = [torch.empty_like(packed) for _ in range(world)]
    dist.all_gather(out, packed, group=group)
    allp = torch.stack(out, dim=1)  # [nq, world, k, 2]
    d = allp[..., 0].to(torch.int32).view(torch.float32)
    r = allp[..., 1]
    return d.contiguous(), r.contiguous()


def sharded_search(engine, shard, queries: torch.Tensor, metric: int, k: int,
                   group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Local fused scan on this rank's shard, all-gather, deterministic merge.

    ``shard.row_base`` must be the shard's first global row (``shard_rows``),
    so the merged rows are positions in the concatenated table.  Over a gloo
    group (CPU tests, several ranks sharing one GPU) the k lists travel
    through host memory; over RCCL they stay on the device."""
    d_loc, r_loc = engine.search([shard], queries, metric, k)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return d_loc, r_loc
    if dist.get_backend(group) == "gloo" and d_loc.is_cuda:
        dev = d_loc.device
        d_all, r_all = allgather_topk(d_loc.cpu(), r_loc.cpu(), group)
        d_all, r_all = d_all.to(dev), r_all.to(dev)
    else:
        d_all, r_all = allgather_topk(d_loc, r_loc, group)
    with engine.lock:
        return engine.merge(d_all, r_all, k)
