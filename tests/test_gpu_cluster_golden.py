"""The product's GPU clustering path (MFMA cosine affinity, p-pruning + Laplacian kernel,
rocSOLVER eigenpairs) vs fixtures produced by the REFERENCE ``speakerlab/process/cluster.py``
(``tests/golden/make_cluster_golden.py``).  The GPU affinity differs from sklearn's float32
GEMM in the last bits, so labels are compared as partitions (cluster ids relabelled by first
occurrence) and the Laplacian to 2e-6 + 1e-6 relative (the degree diagonal); the host decisions on identical affinities are pinned
bit for bit by ``tests/test_cluster_golden.py``."""
import json
import os

import numpy as np
import pytest
import torch

from speakerlab import _hip
from speakerlab.process import cluster as C

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'cluster_golden.npz'))
NAMES = json.loads(G['names'].tobytes())
SPEC = sorted({k.split('/')[0] for k in G.files if k.startswith('spec_n')})


def canon(labels):
    m = {}
    return [m.setdefault(int(v), len(m)) for v in labels]


@pytest.mark.parametrize('name', NAMES)
def test_common_clustering_gpu_matches_reference(name):
    X = G[f'{name}/X']
    ctor = json.loads(G[f'{name}/ctor'].tobytes())
    call = json.loads(G[f'{name}/call'].tobytes())
    cc = C.CommonClustering(**ctor)
    np.random.seed(int(G[f'{name}/seed']))
    labels = cc(X.copy(), **call)
    assert canon(labels) == G[f'{name}/canon'].tolist()


@pytest.mark.parametrize('key', SPEC)
def test_gpu_laplacian_matches_reference(key):
    X, L = G[f'{key}/X'], G[f'{key}/L']
    _, _, p, m = key.split('_')
    n = X.shape[0]
    S = _hip.cosine_affinity(torch.from_numpy(X).cuda())
    Lg = _hip.spectral_laplacian(S, C.pruned_count(n, float(p[1:]), int(m[1:]))).cpu().numpy()
    np.testing.assert_array_equal(Lg == 0, L == 0)          # the same entries pruned
    np.testing.assert_allclose(Lg, L, rtol=1e-6, atol=2e-6)
    if f'{key}/lambdas' in G.files:
        w, _ = _hip.symmetric_eig(torch.from_numpy(L.copy()).cuda())
        lam = w.cpu().numpy()[:11]
        np.testing.assert_allclose(lam, G[f'{key}/lambdas'], rtol=0, atol=2e-5)
        assert int(np.argmax(np.diff(lam.astype(np.float64)))) + 1 == int(G[f'{key}/num_spk'])
