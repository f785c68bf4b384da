"""Host-side clustering logic (cluster.py:23-239 restated) on affinities computed in the
test with numpy; the GPU affinity kernel itself is covered by tests/test_gpu_affinity.py.
Reference cluster.py is not importable here (fastcluster/umap/hdbscan absent), so label
parity is pinned by known-answer synthetic speakers (canonicalised partitions)."""
import numpy as np
import pytest

from speakerlab.process import cluster as C


def canon(labels):
    m = {}
    return [m.setdefault(l, len(m)) for l in labels]


def speakers(n_spk, per, dim=192, noise=0.25, seed=0):
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((n_spk, dim))
    X = np.concatenate([c + noise * rng.standard_normal((per, dim)) for c in centers]).astype(np.float32)
    truth = np.repeat(np.arange(n_spk), per)
    perm = rng.permutation(len(X))
    return X[perm], truth[perm]


def cos(X):
    Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
    return (Xn @ Xn.T).astype(np.float32)


def test_p_prune_matches_row_loop():
    rng = np.random.default_rng(1)
    A = rng.random((50, 50)).astype(np.float32)
    ref = A.copy()
    n_elems = min(int((1 - 0.05) * 50), 50 - 6)
    for i in range(50):
        ref[i, np.argsort(ref[i])[:n_elems]] = 0
    np.testing.assert_array_equal(C.p_prune(A.copy(), 0.05, 6), ref)


@pytest.mark.parametrize('n_spk', [2, 4])
def test_ahc_recovers_speakers(n_spk):
    X, truth = speakers(n_spk, 10, seed=n_spk)
    labels = C.ahc_labels(cos(X), 0.3)
    assert canon(labels) == canon(truth)


def test_spectral_recovers_speakers():
    np.random.seed(0)
    X, truth = speakers(4, 30, seed=7)
    labels = C.spectral_labels(cos(X), max_num_spks=8, pval=0.1)
    assert canon(labels) == canon(truth)


def test_filter_and_merge():
    cc = C.CommonClustering.__new__(C.CommonClustering)
    cc.min_cluster_size = 2
    X, truth = speakers(2, 6, seed=3)
    labels = truth.copy()
    labels[0] = 7                      # a singleton minor cluster
    out = cc.filter_minor_cluster(labels.copy(), X, 2)
    assert canon(out) == canon(truth)
    merged = cc.merge_by_cos(np.array([0, 1]), np.stack([X[0], X[0] * 1.01]), 0.5)
    assert len(set(merged)) == 1
