"""Clustering back-ends — drop-in for ``speakerlab.process.cluster``
(reference ``speakerlab/process/cluster.py:23-239``).

The N x N cosine affinity, the O(N^2 E) part, runs on the GPU (``spk_cosine_affinity``,
MFMA); the decisions that follow stay on the host exactly as in the reference:

* AHC (``cluster.py:139-156``): condensed(-S) -> average linkage (scipy's NN-chain
  implementation of the same Lance-Williams average linkage the reference gets from
  fastcluster, which is not installed here) -> shift by the minimum -> fcluster -1;
* spectral (``cluster.py:23-112``): per-row p-pruning, symmetrisation, unnormalised
  Laplacian, ARPACK ``eigsh(which='SM')``, eigen-gap, sklearn ``k_means``;
* ``filter_minor_cluster`` / ``merge_by_cos`` (``cluster.py:202-239``) on centroids.

The affinity-consuming steps are exposed as functions of the affinity matrix
(``ahc_labels``, ``spectral_labels``) so they can be reused with row blocks gathered from
several GPUs.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse.linalg
from scipy.cluster.hierarchy import fcluster, linkage
from scipy.spatial.distance import squareform


def cosine_affinity(X) -> np.ndarray:
    """sklearn ``cosine_similarity(X, X)`` semantics (float32), computed on the GPU."""
    import torch
    from speakerlab import _hip
    t = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float32))
    if not torch.cuda.is_available():
        raise _hip.HipError('cosine affinity runs on the ROCm device; none is available')
    return _hip.cosine_affinity(t.cuda()).cpu().numpy()


def _host_cosine(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Small centroid-vs-centroid cosines (a few x a few); same normalisation rule."""
    def nrm(x):
        x = np.asarray(x, dtype=np.float64)
        n = np.linalg.norm(x, axis=1, keepdims=True)
        n[n == 0] = 1.0
        return x / n
    return nrm(a) @ nrm(b).T


def ahc_labels(S: np.ndarray, fix_cos_thr: float) -> np.ndarray:
    """AHC on a cosine affinity matrix (cluster.py:149-156)."""
    dist = squareform(-np.asarray(S), checks=False)
    lin = linkage(dist, method='average')
    adjust = abs(lin[:, 2].min())
    lin[:, 2] += adjust
    return fcluster(lin, -fix_cos_thr + adjust, criterion='distance') - 1


def pruned_count(n: int, pval: float, min_pnum: int) -> int:
    """Entries zeroed per row by ``p_pruning`` (cluster.py:67-73): the reference slices
    ``argsort(row)[0:n_elems]`` with ``n_elems = min(int((1 - pval) * n), n - min_pnum)``, so a
    negative n_elems (n < min_pnum) zeroes all but the |n_elems| largest entries, and a count
    past n zeroes the whole row -- Python slice semantics, reproduced here."""
    n_elems = min(int((1 - pval) * n), n - min_pnum)
    return len(range(n)[0:n_elems])


def p_prune(A: np.ndarray, pval: float, min_pnum: int) -> np.ndarray:
    """Zero the smallest entries of every row (cluster.py:64-77), vectorised (stable sort:
    ties go lowest index first, like the GPU kernel)."""
    cnt = pruned_count(A.shape[0], pval, min_pnum)
    if cnt > 0:
        low = np.argsort(A, axis=1, kind='stable')[:, :cnt]
        np.put_along_axis(A, low, 0, axis=1)
    return A


def laplacian(S: np.ndarray, pval: float, min_pnum: int) -> np.ndarray:
    """p-pruning -> 0.5 (A + A^T) -> zero diagonal -> D - A (cluster.py:43-49, 64-84)."""
    A = p_prune(np.array(S, copy=True), pval, min_pnum)
    A = 0.5 * (A + A.T)
    np.fill_diagonal(A, 0)
    return np.diag(np.abs(A).sum(axis=1)) - A


def spectral_labels(S: np.ndarray, min_num_spks=1, max_num_spks=10, pval=0.02, min_pnum=6, oracle_num=None):
    """Spectral clustering of a cosine affinity matrix (cluster.py:35-112)."""
    from sklearn.cluster._kmeans import k_means
    L = laplacian(S, pval, min_pnum)
    lambdas, vecs = scipy.sparse.linalg.eigsh(L, k=min(max_num_spks + 1, L.shape[0]), which='SM')
    if oracle_num is not None:
        k = oracle_num
    else:
        gaps = np.diff(lambdas[min_num_spks - 1:max_num_spks + 1].astype(np.float64))
        k = int(np.argmax(gaps)) + min_num_spks
    _, labels, _ = k_means(vecs[:, :k], k)
    return labels


_solver_warm = False


def _warm_solver():
    """rocBLAS / rocSOLVER load their kernels on first use (~1 s): pay it at construction."""
    global _solver_warm
    if _solver_warm:
        return
    import torch
    if torch.cuda.is_available():
        from speakerlab import _hip
        _hip.symmetric_eig(torch.eye(8, device='cuda'))
        _solver_warm = True


def spectral_labels_gpu(X, min_num_spks=1, max_num_spks=10, pval=0.02, min_pnum=6, oracle_num=None):
    """The same steps with the N x N work on the GPU: cosine affinity (MFMA), p-pruning +
    symmetrisation + Laplacian (csrc/spectral.hip), all eigenpairs by rocSOLVER ssyevd (in
    place of ARPACK eigsh 'SM'); eigen-gap and k-means on the host as in the reference."""
    import torch
    from speakerlab import _hip
    if not torch.cuda.is_available():
        raise _hip.HipError('spectral clustering runs on the ROCm device; none is available')
    t = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float32)).cuda()
    return spectral_labels_gpu_affinity(_hip.cosine_affinity(t), min_num_spks, max_num_spks, pval, min_pnum,
                                        oracle_num)


def spectral_labels_gpu_affinity(S, min_num_spks=1, max_num_spks=10, pval=0.02, min_pnum=6, oracle_num=None):
    """spectral_labels_gpu from a cosine affinity already on the device (e.g. row blocks
    gathered from several GPUs, ``bin/infer_diarization.py --shard_chunks``)."""
    import torch
    from sklearn.cluster._kmeans import k_means
    from speakerlab import _hip
    S = torch.as_tensor(S).to('cuda', torch.float32).contiguous()
    n = S.shape[0]
    L = _hip.spectral_laplacian(S, pruned_count(n, pval, min_pnum))
    del S
    kk = min(max_num_spks + 1, n)
    w, V = _hip.symmetric_eig(L)
    lambdas = w[:kk].cpu().numpy()
    if oracle_num is not None:
        k = oracle_num
    else:
        gaps = np.diff(lambdas[min_num_spks - 1:max_num_spks + 1].astype(np.float64))
        k = int(np.argmax(gaps)) + min_num_spks
    emb = V[:k].t().contiguous().cpu().numpy()
    _, labels, _ = k_means(emb, k)
    return labels


class SpectralCluster:
    def __init__(self, min_num_spks=1, max_num_spks=10, pval=0.02, min_pnum=6, oracle_num=None):
        self.min_num_spks, self.max_num_spks = min_num_spks, max_num_spks
        self.min_pnum, self.pval, self.k = min_pnum, pval, oracle_num
        _warm_solver()

    def __call__(self, X, **kwargs):
        pval = kwargs.get('pval', None)
        oracle = kwargs.get('speaker_num', None)
        return spectral_labels_gpu(X, self.min_num_spks, self.max_num_spks, self.pval if pval is None else pval,
                                   self.min_pnum, self.k if oracle is None else oracle)

    def from_affinity(self, S, **kwargs):
        pval = kwargs.get('pval', None)
        oracle = kwargs.get('speaker_num', None)
        return spectral_labels_gpu_affinity(S, self.min_num_spks, self.max_num_spks,
                                            self.pval if pval is None else pval, self.min_pnum,
                                            self.k if oracle is None else oracle)


class UmapHdbscan:
    """Optional back-end of the reference (umap-learn + hdbscan); not installed here."""

    def __init__(self, n_neighbors=20, n_components=60, min_samples=20, min_cluster_size=10, metric='euclidean'):
        try:
            import hdbscan  # noqa: F401
            import umap  # noqa: F401
        except ImportError as e:
            raise ImportError('Package "umap" or "hdbscan" not found. Please install them first by '
                              '"pip install umap-learn hdbscan".') from e
        self.kw = dict(n_neighbors=n_neighbors, n_components=n_components, min_samples=min_samples,
                       min_cluster_size=min_cluster_size, metric=metric)

    def __call__(self, X, **kwargs):
        import hdbscan
        import umap
        k = self.kw
        emb = umap.UMAP(n_neighbors=k['n_neighbors'], min_dist=0.0, n_components=min(k['n_components'], X.shape[0] - 2),
                        metric=k['metric']).fit_transform(X)
        return hdbscan.HDBSCAN(min_samples=k['min_samples'], min_cluster_size=k['min_cluster_size']).fit_predict(emb)


class AHCluster:
    def __init__(self, fix_cos_thr=0.4):
        self.fix_cos_thr = fix_cos_thr

    def __call__(self, X, **kwargs):
        return ahc_labels(cosine_affinity(X), self.fix_cos_thr)

    def from_affinity(self, S, **kwargs):
        return ahc_labels(S.cpu().numpy() if hasattr(S, 'cpu') else np.asarray(S), self.fix_cos_thr)


class CommonClustering:
    """Dispatch (N < cluster_line -> AHC), then minor-cluster filtering and centroid merging."""

    def __init__(self, cluster_type, cluster_line=40, mer_cos=None, min_cluster_size=4, **kwargs):
        self.cluster_type, self.cluster_line = cluster_type, cluster_line
        self.min_cluster_size, self.mer_cos = min_cluster_size, mer_cos
        if cluster_type == 'spectral':
            self.cluster = SpectralCluster(**kwargs)
        elif cluster_type == 'umap_hdbscan':
            kwargs['min_cluster_size'] = min_cluster_size
            self.cluster = UmapHdbscan(**kwargs)
        elif cluster_type == 'AHC':
            self.cluster = AHCluster(**kwargs)
        else:
            raise ValueError('%s is not currently supported.' % cluster_type)
        self.cluster_for_short = self.cluster if cluster_type == 'AHC' else AHCluster()

    def __call__(self, X, **kwargs):
        assert len(X.shape) == 2, 'Shape of input should be [N, C]'
        if X.shape[0] <= 1:
            return np.zeros(X.shape[0], dtype=int)
        if X.shape[0] < self.cluster_line:
            labels = self.cluster_for_short(X)
        else:
            labels = self.cluster(X, **kwargs)
        return self._finish(labels, X)

    def from_affinity(self, X, S, **kwargs):
        """__call__ with the N x N cosine affinity of X given (e.g. assembled from the row
        blocks several GPUs computed): the same dispatch, clustering and post-processing."""
        assert len(X.shape) == 2 and S.shape[0] == S.shape[1] == X.shape[0]
        if X.shape[0] <= 1:
            return np.zeros(X.shape[0], dtype=int)
        if X.shape[0] < self.cluster_line or not hasattr(self.cluster, 'from_affinity'):
            if X.shape[0] >= self.cluster_line:   # a back-end without an affinity form (umap_hdbscan)
                labels = self.cluster(X, **kwargs)
            else:
                labels = self.cluster_for_short.from_affinity(S)
        else:
            labels = self.cluster.from_affinity(S, **kwargs)
        return self._finish(labels, X)

    def _finish(self, labels, X):
        labels = self.filter_minor_cluster(labels, X, self.min_cluster_size)
        if self.mer_cos is not None:
            labels = self.merge_by_cos(labels, X, self.mer_cos)
        return labels

    def filter_minor_cluster(self, labels, x, min_cluster_size):
        cset, csize = np.unique(labels, return_counts=True)
        minor = cset[csize <= self.min_cluster_size]
        if len(minor) == 0:
            return labels
        major = cset[csize > self.min_cluster_size]
        if len(major) == 0:
            return np.zeros_like(labels)
        centers = np.stack([x[labels == c].mean(0) for c in major])
        for i in np.nonzero(np.isin(labels, minor))[0]:
            labels[i] = major[_host_cosine(x[i][None], centers).argmax()]
        return labels

    def merge_by_cos(self, labels, x, cos_thr):
        assert 0 < cos_thr <= 1
        while True:
            cset = np.unique(labels)
            if len(cset) == 1:
                break
            centers = np.stack([x[labels == c].mean(0) for c in cset])
            aff = np.triu(_host_cosine(centers, centers), 1)
            i, j = np.unravel_index(np.argmax(aff), aff.shape)
            if aff[i, j] < cos_thr:
                break
            labels[labels == cset[j]] = cset[i]
        return labels
