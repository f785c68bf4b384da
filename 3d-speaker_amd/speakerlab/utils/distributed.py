"""Process-per-GPU sharding + the one collective of the path.

The reference shards utterances ``wav_list[rank::nprocs]`` with no process group and
writes files (``infer_sv_batch.py:348-350``, ``infer_diarization.py:924``).  Here the shard
is a contiguous block (keeps output order and locality), and scoring gathers every
rank's embeddings with ONE all-gather (RCCL over xGMI when the backend is ``nccl``),
after which each rank scores its own row block of the N x N cosine affinity with the
MFMA kernel — the full matrix is never materialised on one device.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [start, stop) of ceil(n / world) items for ``rank``."""
    per = math.ceil(n / world) if world > 0 else n
    start = min(n, rank * per)
    return start, min(n, start + per)


def all_gather_embeddings(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Gather every rank's [n_local, E] block (contiguous sharding of ``n_total`` rows) into
    [n_total, E] on every rank.  Uneven shards are padded to ceil(n_total/world) rows."""
    world = dist.get_world_size(group)
    per = math.ceil(n_total / world)
    E = local.shape[1]
    padded = torch.zeros((per, E), dtype=local.dtype, device=local.device)
    padded[:local.shape[0]] = local
    if dist.get_backend(group) == 'nccl':
        out = torch.empty((world * per, E), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, padded, group=group)
        blocks = out.view(world, per, E)
    else:
        parts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(parts, padded, group=group)
        blocks = torch.stack(parts)
    rows = []
    for r in range(world):
        s, e = shard_bounds(n_total, r, world)
        rows.append(blocks[r, :e - s])
    return torch.cat(rows, 0)


def all_gather_rows(local: torch.Tensor, counts, group=None) -> torch.Tensor:
    """Concatenate every rank's [counts[r], ...] block in rank order on every rank (blocks of
    unequal size are padded to max(counts) for the collective).  nccl gathers device tensors
    with one ``all_gather_into_tensor``; gloo gathers host copies."""
    world = dist.get_world_size(group)
    assert len(counts) == world and local.shape[0] == counts[dist.get_rank(group)]
    per = max(max(counts), 1)
    nccl = dist.get_backend(group) == 'nccl'
    src = local if nccl else local.cpu()
    padded = torch.zeros((per,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    padded[:src.shape[0]] = src
    if nccl:
        out = torch.empty((world * per,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        dist.all_gather_into_tensor(out, padded, group=group)
        blocks = out.view((world, per) + tuple(src.shape[1:]))
    else:
        parts = [torch.empty_like(padded) for _ in range(world)]
        dist.all_gather(parts, padded, group=group)
        blocks = torch.stack(parts)
    return torch.cat([blocks[r, :counts[r]] for r in range(world)], 0).to(local.device)


def batch_shard(n: int, batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [start, stop) of WHOLE batches of ``batch`` items for ``rank``: every
    rank runs exactly the batches a single process would run (same batch composition, hence
    bitwise the same per-row results as one process)."""
    nb = math.ceil(n / batch) if batch > 0 else 0
    b0, b1 = shard_bounds(nb, rank, world)
    return min(n, b0 * batch), min(n, b1 * batch)


def affinity_row_block(emb_all: torch.Tensor, rank: int, world: int, out: Optional[torch.Tensor] = None):
    """(row0, [rows, N]) cosine affinity of this rank's rows against all N embeddings,
    computed on the GPU by ``spk_cosine_affinity``."""
    from speakerlab import _hip
    s, e = shard_bounds(emb_all.shape[0], rank, world)
    return s, _hip.cosine_affinity(emb_all[s:e], emb_all, out=out)


def topk_row_block(emb_all: torch.Tensor, rank: int, world: int, k: int = 1, threshold: float = float('inf')):
    """This rank's row block consumed in place: for each of its rows the k best matches among
    all N embeddings (self excluded) and the count of scores >= threshold (``spk_cosine_topk``;
    the row block of the affinity is never written).  Returns (row0, scores, index, count)."""
    from speakerlab import _hip
    s, e = shard_bounds(emb_all.shape[0], rank, world)
    sc, ix, cnt = _hip.cosine_topk(emb_all[s:e], emb_all, k=k, self_offset=s, threshold=threshold)
    return s, sc, ix, cnt
