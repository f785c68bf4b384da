"""GPU spectral clustering pieces vs the reference's host algorithm
(speakerlab/process/cluster.py:64-105): p-pruning + Laplacian kernel, rocSOLVER eigenpairs,
and the resulting labels."""
import numpy as np
import pytest
import torch

from speakerlab import _hip
from speakerlab.process import cluster

pytestmark = pytest.mark.gpu


def _ref_laplacian(S, pval, min_pnum):
    """The reference's loops (cluster.py:64-84) on a float32 copy."""
    A = S.copy()
    n = A.shape[0]
    n_elems = min(int((1 - pval) * n), n - min_pnum)
    for i in range(n):
        A[i, np.argsort(A[i, :])[:n_elems]] = 0
    M = 0.5 * (A + A.T)
    M[np.diag_indices(n)] = 0
    return np.diag(np.sum(np.abs(M), axis=1)) - M, n_elems


@pytest.mark.parametrize('n', [7, 300, 1500])
def test_laplacian_kernel_matches_reference_loops(n):
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, 192)).astype(np.float32)
    S = _hip.cosine_affinity(torch.from_numpy(X).cuda())
    Sh = S.cpu().numpy()
    ref, n_elems = _ref_laplacian(Sh, 0.02 if n > 100 else 0.2, 6 if n > 10 else 2)
    L = _hip.spectral_laplacian(S, n_elems).cpu().numpy()
    off = ~np.eye(n, dtype=bool)
    np.testing.assert_array_equal(L[off], ref[off])                       # exact (no ties in random data)
    np.testing.assert_allclose(np.diag(L), np.diag(ref), rtol=2e-5, atol=1e-6)


def test_pruning_ties_lowest_index_first():
    S = torch.tensor([[1.0, 0.5, 0.5, 0.5, 0.2], [0.5, 1.0, 0.5, 0.5, 0.5], [0.5, 0.5, 1.0, 0.5, 0.5],
                      [0.5, 0.5, 0.5, 1.0, 0.5], [0.2, 0.5, 0.5, 0.5, 1.0]], device='cuda')
    L = _hip.spectral_laplacian(S, 2).cpu().numpy()
    # row 0: 0.2 (index 4) and the lowest-index 0.5 (index 1) pruned; symmetrised with row 1
    # (which prunes indices 0 and 2)
    M = -L.copy()
    np.fill_diagonal(M, 0)
    assert M[0, 1] == 0.0 and M[0, 4] == pytest.approx(0.5 * (0.0 + 0.0)) and M[0, 2] == pytest.approx(0.5 * (0.5 + 0.0))


def test_symmetric_eig():
    rng = np.random.default_rng(1)
    B = rng.standard_normal((200, 200)).astype(np.float32)
    A = (B + B.T) / 2
    w, V = _hip.symmetric_eig(torch.from_numpy(A.copy()).cuda())
    w, V = w.cpu().numpy(), V.cpu().numpy()
    ref = np.linalg.eigvalsh(A.astype(np.float64))
    np.testing.assert_allclose(w, ref, rtol=1e-4, atol=1e-4)
    resid = np.abs(A @ V.T - V.T * w[None]).max()
    assert resid < 1e-3, resid


@pytest.mark.parametrize('n,k', [(240, 3), (900, 5)])
def test_spectral_labels_match_host_reference(n, k):
    rng = np.random.default_rng(k)
    centers = rng.standard_normal((k, 192))
    truth = rng.integers(0, k, n)
    X = (centers[truth] + 0.3 * rng.standard_normal((n, 192))).astype(np.float32)
    np.random.seed(0)
    gpu = cluster.spectral_labels_gpu(X, max_num_spks=8, pval=0.05)
    S = cluster.cosine_affinity(X)
    np.random.seed(0)
    host = cluster.spectral_labels(S, max_num_spks=8, pval=0.05)

    def canon(v):
        m = {}
        return [m.setdefault(x, len(m)) for x in v]
    assert canon(gpu) == canon(host) == canon(truth)
