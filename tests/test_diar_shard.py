"""C5 on several ranks: ONE meeting's chunks sharded across a process group
(`infer_diarization.py --shard_chunks`) -- whole embedding batches per rank, one all-gather of
the embeddings, a row block of the cosine affinity per rank, gathered for the clustering --
must give exactly the single-process result: the same embeddings bit for bit, the same
affinity, the same labels and RTTM.  CPU, gloo, world size 2: the GPU embedding model and
affinity kernel are replaced by deterministic host stand-ins of the same shapes (their GPU
parity is `test_gpu_diarization.py`'s); the sharding, gathers and clustering dispatch are the
product code."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from speakerlab.bin import infer_diarization as idz
from speakerlab.process import cluster as cl
from speakerlab.utils.distributed import all_gather_rows, batch_shard


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Feat:
    """Stand-in Fbank: log power spectrum of 160-sample frames (80 bins)."""
    sample_rate = 16000

    def batch(self, w):
        T = w.shape[1] // 160
        spec = torch.fft.rfft(w[:, :T * 160].reshape(w.shape[0], T, 160).double(), dim=-1)
        return torch.log(spec.abs()[:, :, 1:81] ** 2 + 1e-6).float()


class _Emb(torch.nn.Module):
    """Stand-in embedding model: the time-averaged log spectrum, centred over the bins, so
    chunks of one synthetic speaker (one carrier frequency) point the same way."""
    embedding_size = 80

    def forward(self, f):
        m = f.mean(1)
        return m - m.mean(1, keepdim=True)


def _host_affinity(a, b=None):
    """cosine similarity in float64, rounded once: a row block equals the rows of the whole"""
    b = a if b is None else b
    a, b = a.double(), b.double()
    an = a / a.norm(dim=1, keepdim=True).clamp_min(1e-12)
    bn = b / b.norm(dim=1, keepdim=True).clamp_min(1e-12)
    return (an @ bn.t()).float()


def _diar(group, cluster_type):
    d = object.__new__(idz.Diarization3Dspeaker)
    d.device = torch.device('cpu')
    d.feature_extractor = _Feat()
    d.embedding_model = _Emb()
    d.batchsize = 8
    d.fs = 16000
    d.speaker_num = None
    d.group = group
    kw = {'cluster_line': 10} if cluster_type == 'spectral' else {}
    d.cluster = object.__new__(cl.CommonClustering)
    d.cluster.cluster_type, d.cluster.cluster_line = cluster_type, kw.get('cluster_line', 40)
    d.cluster.min_cluster_size, d.cluster.mer_cos = 0, 0.3
    if cluster_type == 'spectral':
        sc = object.__new__(cl.SpectralCluster)
        sc.min_num_spks, sc.max_num_spks, sc.min_pnum, sc.pval, sc.k = 1, 10, 6, 0.02, None
        d.cluster.cluster = sc
    else:
        d.cluster.cluster = cl.AHCluster(0.3)
    d.cluster.cluster_for_short = cl.AHCluster()
    return d


def _meeting(n_spk=3, seconds=40, seed=3):
    """Synthetic meeting: speaker turns of 2-4 s, each speaker a carrier of its own frequency."""
    rng = np.random.default_rng(seed)
    fs = 16000
    w = np.zeros(seconds * fs, np.float32)
    t, chunks = 0.0, []
    while t < seconds - 1:
        dur = min(float(rng.uniform(2, 4)), seconds - t)
        spk = int(rng.integers(n_spk))
        a, b = int(t * fs), int((t + dur) * fs)
        tt = np.arange(b - a) / fs
        x = 0.05 * rng.standard_normal(b - a) + np.sin(2 * np.pi * (1000 + 1700 * spk) * tt)
        w[a:b] = x.astype(np.float32)
        chunks += [[st, ed] for st, ed in _chunks(t, t + dur)]
        t += dur
    return torch.from_numpy(w)[None], chunks


def _chunks(st, ed, dur=1.5, step=0.75):
    out, s = [], st
    while s + dur < ed:
        out.append([round(s, 3), round(s + dur, 3)])
        s += step
    out.append([round(max(st, ed - dur), 3), round(ed, 3)])
    return out


def _run(group, cluster_type):
    wav, chunks = _meeting()
    d = _diar(group, cluster_type)
    emb = d.do_emb_extraction(chunks, wav)
    np.random.seed(0)    # sklearn k_means draws its centroids from numpy's global RNG (reference)
    spk, segs = d.do_clustering(chunks, emb)
    return emb, spk, segs


def _patch():
    # host stand-ins of the GPU kernels the clustering would call
    import speakerlab._hip as hip
    hip.cosine_affinity = lambda a, b=None, out=None: _host_affinity(a, b)
    cl.cosine_affinity = lambda X: _host_affinity(torch.as_tensor(np.asarray(X, np.float32))).numpy()

    def spec_aff(S, mn=1, mx=10, pval=0.02, min_pnum=6, oracle_num=None):
        return cl.spectral_labels(np.asarray(S.cpu() if hasattr(S, 'cpu') else S, np.float64), mn, mx, pval,
                                  min_pnum, oracle_num)
    cl.spectral_labels_gpu_affinity = spec_aff
    cl.spectral_labels_gpu = lambda X, *a: spec_aff(_host_affinity(torch.as_tensor(np.asarray(X, np.float32))), *a)


def _worker(rank, world, port, cluster_type, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        _patch()
        emb, spk, segs = _run(dist.group.WORLD, cluster_type)
        q.put((rank, emb, int(spk), segs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('cluster_type', ['AHC', 'spectral'])
def test_shard_chunks_two_ranks_equals_one_process(cluster_type):
    _patch()
    emb1, spk1, segs1 = _run(None, cluster_type)
    assert spk1 >= 2, 'the synthetic meeting should separate into several speakers'
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cluster_type, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, emb, spk, segs = q.get(timeout=180)
        res[r] = (emb, spk, segs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        emb, spk, segs = res[r]
        assert np.array_equal(emb, emb1), r          # bitwise: each rank runs whole single-process batches
        assert spk == spk1 and segs == segs1, r      # same labels -> the same RTTM lines


def test_batch_shard_whole_batches():
    for n in (1, 7, 64, 65, 3538):
        for bs in (1, 8, 64):
            for w in (1, 2, 3, 8):
                spans = [batch_shard(n, bs, r, w) for r in range(w)]
                assert spans[0][0] == 0 and spans[-1][1] == n
                assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
                assert all(s % bs == 0 for s, _ in spans if s < n)


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        counts = [5, 0, 3][:world]
        full = torch.arange(sum(counts) * 3, dtype=torch.float32).view(-1, 3)
        s = sum(counts[:rank])
        got = all_gather_rows(full[s:s + counts[rank]].clone(), counts)
        q.put((rank, bool(torch.equal(got, full))))
    finally:
        dist.destroy_process_group()


def test_all_gather_rows_uneven_three_ranks():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True, 2: True}
