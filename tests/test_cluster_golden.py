"""Clustering host logic vs fixtures produced by the REFERENCE ``speakerlab/process/cluster.py``
(``tests/golden/make_cluster_golden.py``: the reference module imported read-only with
``fastcluster.linkage`` -> scipy ``linkage`` as the one stand-in).  The affinity is sklearn's
``cosine_similarity`` here (the reference's own call, cluster.py:61,150), so these tests pin the
host decisions exactly; ``tests/test_gpu_cluster_golden.py`` runs the same fixtures through the
GPU affinity / Laplacian / eigensolver path."""
import json
import os

import numpy as np
import pytest
from sklearn.metrics.pairwise import cosine_similarity

from speakerlab.process import cluster as C

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'cluster_golden.npz'))
NAMES = json.loads(G['names'].tobytes())
SPEC = sorted({k.split('/')[0] for k in G.files if k.startswith('spec_n')})


def canon(labels):
    m = {}
    return [m.setdefault(int(v), len(m)) for v in labels]


def case(name):
    return (G[f'{name}/X'], json.loads(G[f'{name}/ctor'].tobytes()), json.loads(G[f'{name}/call'].tobytes()),
            int(G[f'{name}/seed']))


class _HostSpectral(C.SpectralCluster):
    """The product's host spectral path (the product class runs the GPU path)."""

    def __call__(self, X, **kw):
        pval = kw.get('pval', None)
        oracle = kw.get('speaker_num', None)
        return C.spectral_labels(cosine_similarity(X, X), self.min_num_spks, self.max_num_spks,
                                 self.pval if pval is None else pval, self.min_pnum,
                                 self.k if oracle is None else oracle)


@pytest.fixture
def host_backends(monkeypatch):
    monkeypatch.setattr(C, 'cosine_affinity', lambda X: cosine_similarity(X))
    monkeypatch.setattr(C, '_warm_solver', lambda: None)
    monkeypatch.setattr(C, 'SpectralCluster', _HostSpectral)


@pytest.mark.parametrize('name', NAMES)
def test_common_clustering_matches_reference(name, host_backends):
    X, ctor, call, seed = case(name)
    cc = C.CommonClustering(**ctor)
    np.random.seed(seed)
    labels = cc(X.copy(), **call)
    # same affinity bits, same linkage / eigsh / k_means under the same seed: the raw labels
    # are the reference's, not only the partition
    np.testing.assert_array_equal(labels, G[f'{name}/labels'])


@pytest.mark.parametrize('key', SPEC)
def test_laplacian_matches_reference(key):
    X, L = G[f'{key}/X'], G[f'{key}/L']
    _, _, p, m = key.split('_')
    Lp = C.laplacian(cosine_similarity(X, X), float(p[1:]), int(m[1:]))
    np.testing.assert_array_equal(Lp.astype(np.float32), L)


@pytest.mark.parametrize('key', [k for k in SPEC if f'{k}/lambdas' in G.files])
def test_eigen_gap_matches_reference(key):
    import scipy.sparse.linalg
    lam, _ = scipy.sparse.linalg.eigsh(G[f'{key}/L'], k=11, which='SM')
    np.testing.assert_allclose(lam, G[f'{key}/lambdas'], rtol=1e-4, atol=1e-5)
    gaps = np.diff(lam[0:11].astype(np.float64))
    assert int(np.argmax(gaps)) + 1 == int(G[f'{key}/num_spk'])


@pytest.mark.parametrize('n,pval,min_pnum,expect', [(50, 0.02, 6, 44), (6, 0.02, 8, 4), (9, 0.02, 12, 6),
                                                     (3, 0.02, 6, 0), (40, 0.5, 30, 10), (100, -0.5, 0, 100)])
def test_pruned_count_slice_semantics(n, pval, min_pnum, expect):
    assert C.pruned_count(n, pval, min_pnum) == expect
    n_elems = min(int((1 - pval) * n), n - min_pnum)
    assert C.pruned_count(n, pval, min_pnum) == len(np.argsort(np.arange(n))[0:n_elems])


def test_filter_minor_cluster_matches_reference():
    cc = C.CommonClustering.__new__(C.CommonClustering)
    cc.min_cluster_size = 4
    out = cc.filter_minor_cluster(G['filter/in'].copy(), G['filter/X'], 4)
    np.testing.assert_array_equal(out, G['filter/out'])


@pytest.mark.parametrize('thr', [0.3, 0.8, 0.95])
def test_merge_by_cos_matches_reference(thr):
    cc = C.CommonClustering.__new__(C.CommonClustering)
    out = cc.merge_by_cos(G['merge/in'].copy(), G['merge/X'], thr)
    np.testing.assert_array_equal(out, G[f'merge/out_{thr}'])
