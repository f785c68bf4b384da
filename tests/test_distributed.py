"""Multi-process path on CPU (gloo, world_size 2): contiguous sharding and the embedding
all-gather used before the row-block affinity."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from speakerlab.utils.distributed import all_gather_embeddings, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        full = torch.arange(n_total * 6, dtype=torch.float32).view(n_total, 6)
        s, e = shard_bounds(n_total, rank, world)
        got = all_gather_embeddings(full[s:e].clone(), n_total)
        q.put((rank, bool(torch.equal(got, full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('n_total', [8, 7, 1])
def test_all_gather_two_ranks(n_total):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 100, 100000):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
