"""Consumers of the cosine affinity behind the C ABI: row-block top-k with
self exclusion and threshold counts (``spk_cosine_topk``), and the per-trial gather of
``compute_score_metrics.py:102-118`` (``spk_cosine_trials``), checked against float64 numpy
cosines (sklearn ``cosine_similarity`` semantics)."""
import numpy as np
import pytest
import torch

from speakerlab import _hip

pytestmark = pytest.mark.gpu


def np_cos(a, b):
    def nrm(x):
        x = x.astype(np.float64)
        n = np.linalg.norm(x, axis=1, keepdims=True)
        n[n == 0] = 1.0
        return x / n
    return nrm(a) @ nrm(b).T


def np_topk(S, k, self_off):
    S = S.copy()
    if self_off is not None:
        r = np.arange(S.shape[0])
        ok = r + self_off < S.shape[1]
        S[r[ok], r[ok] + self_off] = -np.inf
    order = np.lexsort((np.broadcast_to(np.arange(S.shape[1]), S.shape), -S), axis=1)[:, :k]
    return np.take_along_axis(S, order, 1), order


@pytest.mark.parametrize('na,nb,e,k,self_off', [(300, 1000, 192, 1, 0), (129, 5000, 192, 8, 100), (1, 7, 512, 5, None),
                                                (2000, 300, 192, 3, None), (513, 40000, 192, 4, 20000)])
def test_topk_matches_numpy(na, nb, e, k, self_off):
    rng = np.random.default_rng(na + nb)
    B = rng.standard_normal((nb, e)).astype(np.float32)
    if self_off is None:
        A = rng.standard_normal((na, e)).astype(np.float32)
    else:
        A = B[self_off:self_off + na].copy()
    A[0] = 0.0                                                  # zero-norm row: sklearn divides by 1
    S = np_cos(A, B)
    thr = 0.1
    sc, ix, cnt = _hip.cosine_topk(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(), k=k,
                                   self_offset=self_off, threshold=thr)
    sc, ix, cnt = sc.cpu().numpy(), ix.cpu().numpy(), cnt.cpu().numpy()
    rs, ri = np_topk(S, min(k, nb), self_off)
    np.testing.assert_allclose(sc[:, :rs.shape[1]], rs, rtol=0, atol=2e-6)
    # indices agree wherever the float64 scores are not within rounding of each other
    gap = np.abs(np.diff(np.concatenate([rs, np.full((na, 1), -np.inf)], 1), axis=1))[:, :rs.shape[1]]
    sure = gap > 1e-5
    np.testing.assert_array_equal(ix[:, :ri.shape[1]][sure], ri[sure])
    Sx = S.copy()
    if self_off is not None:
        r = np.arange(na)
        Sx[r, r + self_off] = -np.inf
    near = np.abs(Sx - thr) < 1e-5
    exact = (Sx >= thr).sum(1)
    assert np.all(np.abs(cnt - exact) <= near.sum(1))


def test_topk_ties_lowest_index_first():
    v = np.zeros((6, 192), dtype=np.float32)
    v[:, 0] = 1.0                                               # six identical rows: all scores 1
    sc, ix, _ = _hip.cosine_topk(torch.from_numpy(v[:2]).cuda(), torch.from_numpy(v).cuda(), k=4, self_offset=0)
    assert ix.cpu().tolist() == [[1, 2, 3, 4], [0, 2, 3, 4]]
    assert np.allclose(sc.cpu().numpy(), 1.0)


def test_topk_fewer_columns_than_k():
    A = np.eye(3, 8, dtype=np.float32)
    sc, ix, _ = _hip.cosine_topk(torch.from_numpy(A).cuda(), torch.from_numpy(A[:2]).cuda(), k=4)
    ix = ix.cpu().numpy()
    assert (ix[:, 2:] == -1).all() and ix[0, 0] == 0 and ix[1, 0] == 1


@pytest.mark.parametrize('e', [192, 512, 80])
def test_trials_match_numpy(e):
    rng = np.random.default_rng(e)
    A = rng.standard_normal((50, e)).astype(np.float32)
    B = rng.standard_normal((70, e)).astype(np.float32)
    B[3] = 0
    ia = rng.integers(0, 50, 5000)
    ib = rng.integers(0, 70, 5000)
    got = _hip.cosine_trials(torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda(), torch.from_numpy(ia),
                             torch.from_numpy(ib)).cpu().numpy()
    np.testing.assert_allclose(got, np_cos(A, B)[ia, ib], rtol=0, atol=2e-6)


def test_trials_reject_out_of_range():
    A = torch.zeros((2, 192), device='cuda')
    with pytest.raises(_hip.HipError):
        _hip.cosine_trials(A, A, torch.tensor([0, 2]), torch.tensor([0, 1]))
