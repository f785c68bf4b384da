"""GPU cosine affinity vs numpy (sklearn cosine_similarity semantics)."""
import numpy as np
import pytest
import torch

from speakerlab import _hip

pytestmark = pytest.mark.gpu


def ref_cos(a, b):
    def norm(x):
        n = np.linalg.norm(x, axis=1, keepdims=True)
        n[n == 0] = 1.0
        return x / n
    return norm(a.astype(np.float64)) @ norm(b.astype(np.float64)).T


@pytest.mark.parametrize('na,nb,e', [(1, 1, 192), (7, 300, 192), (257, 129, 512), (1000, 1000, 192)])
def test_cosine_affinity(na, nb, e):
    rng = np.random.default_rng(na + nb)
    a = rng.standard_normal((na, e)).astype(np.float32)
    b = rng.standard_normal((nb, e)).astype(np.float32)
    a[0] = 0.0   # zero row -> zeros, like sklearn
    out = _hip.cosine_affinity(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    np.testing.assert_allclose(out, ref_cos(a, b), atol=2e-6)


def test_row_blocks_compose_full_matrix():
    """Row-block scoring (one block per rank after the all-gather) == the full matrix."""
    from speakerlab.utils.distributed import affinity_row_block
    rng = np.random.default_rng(3)
    e = torch.from_numpy(rng.standard_normal((1001, 192)).astype(np.float32)).cuda()
    full = _hip.cosine_affinity(e).cpu().numpy()
    blocks = [affinity_row_block(e, r, 3) for r in range(3)]
    stacked = np.concatenate([b.cpu().numpy() for _, b in blocks])
    np.testing.assert_allclose(stacked, full, atol=1e-6)


@pytest.mark.parametrize('ctype,n', [('AHC', 30), ('spectral', 120)])
def test_common_clustering_end_to_end(ctype, n):
    """CommonClustering with the GPU affinity recovers well-separated synthetic speakers."""
    from speakerlab.process.cluster import CommonClustering
    rng = np.random.default_rng(11)
    centers = rng.standard_normal((3, 192))
    truth = np.repeat(np.arange(3), n // 3)
    X = (centers[truth] + 0.25 * rng.standard_normal((n, 192))).astype(np.float32)
    np.random.seed(0)
    kw = dict(pval=0.1, max_num_spks=8) if ctype == 'spectral' else dict(fix_cos_thr=0.3)
    labels = CommonClustering(ctype, mer_cos=0.8, **kw)(X)

    def canon(v):
        m = {}
        return [m.setdefault(x, len(m)) for x in v]
    assert canon(labels) == canon(truth)
