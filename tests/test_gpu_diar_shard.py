"""C5 on the GPU, SURVEY §8(e) row "ERes2NetV2 embed (8 GPU)" and the 1 h clustering scale.

1. One meeting's chunks sharded across two ranks (`Diarization3Dspeaker(group=...)`, the
   `--shard_chunks` CLI path) with the real HIP embedding model and MFMA affinity kernel:
   the gathered embeddings, the affinity assembled from the ranks' row blocks and the output
   segments equal the single-process run bit for bit.  Two gloo ranks share the box's one GPU
   (nccl needs a device per rank; the nccl all-gather itself is `test_gpu_nccl.py`'s).
2. Clustering at C5 scale on an affinity with real structure: N = 3,500 well-separated
   synthetic embeddings (8 speakers) through the GPU spectral path (MFMA affinity,
   p-pruning + Laplacian kernel, rocSOLVER) against the fixture-pinned host decisions
   (`process/cluster.py` laplacian + eigen-gap + k-means, pinned by test_cluster_golden.py)
   on the same affinity: same partition, and it is the true one."""
import os
import socket

import numpy as np
import pytest
import scipy.linalg
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from speakerlab import _hip
from speakerlab.bin import infer_diarization as idz
from speakerlab.process import cluster as C
from speakerlab.utils import synthetic

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(group):
    torch.manual_seed(0)
    wav, _ = synthetic.synth_meeting(60.0, 3, seed=5)
    diar = idz.Diarization3Dspeaker('cuda', synthetic_weights=True, vad='energy', batch_size=16, group=group)
    x = torch.from_numpy(wav)[None]
    flags, xv = diar.do_vad(x)
    _, _, vad_time = diar.postprocess_vad(flags, xv)
    chunks = [c for st, ed in vad_time for c in diar.chunk(st, ed)]
    emb = diar.do_emb_extraction(chunks, x)
    X = torch.from_numpy(emb).cuda()
    if group is None:
        S = _hip.cosine_affinity(X).cpu().numpy()
    else:
        from speakerlab.utils.distributed import all_gather_rows, shard_bounds
        r, w = dist.get_rank(group), dist.get_world_size(group)
        b = [shard_bounds(len(emb), i, w) for i in range(w)]
        S = all_gather_rows(_hip.cosine_affinity(X[b[r][0]:b[r][1]], X), [e - s for s, e in b], group).cpu().numpy()
    np.random.seed(0)
    spk, segs = diar.do_clustering(chunks, emb)
    return emb, S, int(spk), segs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        q.put((rank,) + _run(dist.group.WORLD))
    finally:
        dist.destroy_process_group()


def test_shard_chunks_two_ranks_on_gpu_equal_one_process():
    emb1, S1, spk1, segs1 = _run(None)
    assert len(emb1) > 40          # past cluster_line: the spectral back-end runs
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            r, emb, S, spk, segs = q.get(timeout=240)
            res[r] = (emb, S, spk, segs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in (0, 1):
        emb, S, spk, segs = res[r]
        assert np.array_equal(emb, emb1), r      # whole single-process batches per rank
        assert np.array_equal(S, S1), r          # row blocks of the MFMA affinity == the whole
        assert spk == spk1 and segs == segs1, r


def canon(labels):
    m = {}
    return [m.setdefault(int(v), len(m)) for v in labels]


def test_spectral_c5_scale_separated_speakers():
    rng = np.random.default_rng(11)
    n, k, E = 3500, 8, 192
    centers = rng.standard_normal((k, E))
    truth = rng.integers(0, k, n)
    X = (centers[truth] + 0.45 * rng.standard_normal((n, E))).astype(np.float32)
    np.random.seed(0)
    gpu = C.spectral_labels_gpu(X)
    # host decisions on the same (GPU) affinity: laplacian + eigen-gap + k-means of
    # process/cluster.py, the dense symmetric solver standing in for ARPACK at this size
    S = _hip.cosine_affinity(torch.from_numpy(X).cuda()).cpu().numpy()
    L = C.laplacian(S, 0.02, 6)
    lam, vec = scipy.linalg.eigh(L, subset_by_index=[0, 10])
    gaps = np.diff(lam[0:11].astype(np.float64))
    kk = int(np.argmax(gaps)) + 1
    from sklearn.cluster._kmeans import k_means
    np.random.seed(0)
    _, host, _ = k_means(vec[:, :kk], kk)
    print('C5-scale spectral: N', n, 'speakers found', kk, 'gpu', len(set(gpu)))
    assert kk == k
    assert canon(gpu) == canon(host)
    assert canon(gpu) == canon(truth)
